"""Dataset readers (host side).

* OpenKE benchmark directories (OpenKE/README.md:126-141): `*2id.txt` files whose first line is
  a count and whose rows are `h t r`; `type_constrain.txt` (Reader.h:266-317).
* The zero-shot datasets' test triples (origin_data/{FB15K-237-ZS,DB15K-ZS}/test_tasks_zsl.json
  mapped through entity2ids_zsl.json / relation2ids.json), shipped as compact id arrays under
  mmre/datasets/ (made by mmre/datasets/convert_zs.py in the build container).
"""
from __future__ import annotations

import os

import numpy as np

DATASETS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "datasets")


def read_count(path: str) -> int:
    with open(path) as f:
        return int(f.readline().split()[0])


def read_triples(path: str) -> np.ndarray:
    """(n, 3) int64 rows (h, t, r) as stored in OpenKE files (Reader.h:86-90)."""
    n = read_count(path)
    if n == 0:
        return np.zeros((0, 3), np.int64)
    a = np.loadtxt(path, skiprows=1, dtype=np.int64, ndmin=2)
    return a[:n, :3]


def read_type_constrain(path: str, n_rel: int):
    """type_constrain.txt -> (heads[r], tails[r]) sorted id lists (Reader.h:266-317)."""
    heads = [[] for _ in range(n_rel)]
    tails = [[] for _ in range(n_rel)]
    with open(path) as f:
        toks = f.read().split()
    pos = 1
    for _ in range(n_rel):
        r, n = int(toks[pos]), int(toks[pos + 1])
        heads[r] = sorted(int(x) for x in toks[pos + 2:pos + 2 + n])
        pos += 2 + n
        r, n = int(toks[pos]), int(toks[pos + 1])
        tails[r] = sorted(int(x) for x in toks[pos + 2:pos + 2 + n])
        pos += 2 + n
    return heads, tails


class OpenKEDataset:
    """In-memory view of an OpenKE benchmark directory."""

    def __init__(self, in_path: str, ent_file: str = "", rel_file: str = "", train_file: str = "",
                 valid_file: str = "", test_file: str = ""):
        p = in_path
        self.in_path = p
        self.n_ent = read_count(ent_file or os.path.join(p, "entity2id.txt"))
        self.n_rel = read_count(rel_file or os.path.join(p, "relation2id.txt"))
        self.train = read_triples(train_file or os.path.join(p, "train2id.txt"))
        vf = valid_file or os.path.join(p, "valid2id.txt")
        tf = test_file or os.path.join(p, "test2id.txt")
        self.valid = read_triples(vf) if os.path.exists(vf) else np.zeros((0, 3), np.int64)
        self.test = read_triples(tf) if os.path.exists(tf) else np.zeros((0, 3), np.int64)
        tcp = os.path.join(p, "type_constrain.txt")
        self.type_heads = self.type_tails = None
        if os.path.exists(tcp):
            self.type_heads, self.type_tails = read_type_constrain(tcp, self.n_rel)

    def test_list(self):
        """testList in Test.h order: sorted by (r, h, t) (Reader.h:227, Triple.h:21-23).
        Returns h, r, t int64 arrays."""
        return sorted_rel2(self.test)

    def all_triples(self):
        a = np.concatenate([self.train, self.valid, self.test])
        return a[:, 0], a[:, 2], a[:, 1]


def sorted_rel2(hrt_file_order: np.ndarray):
    a = np.asarray(hrt_file_order, np.int64)
    h, t, r = a[:, 0], a[:, 1], a[:, 2]
    o = np.lexsort((t, h, r))
    return h[o], r[o], t[o]


def load_zs_test(name: str):
    """Zero-shot test triples as id arrays: dict(h, r, t, n_ent, n_rel, rel_names?)."""
    fn = {"FB15K-237-ZS": "fb15k237zs_test.npz", "DB15K-ZS": "db15kzs_test.npz"}[name]
    with np.load(os.path.join(DATASETS_DIR, fn), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


class TrainIndex:
    """The training-triple index of importTrainFiles (Reader.h:53-160), as arrays:

    train_list  unique (h, r, t) rows in cmp_head order (h, r, t)        -- trainList
    head_hrt    same order                                               -- trainHead
    tail_hrt    rows sorted by (t, r, h)                                 -- trainTail
    rel_hrt     rows sorted by (h, t, r)                                 -- trainRel
    lef/rig_*   first / last row of each entity's block (rig = -1 when absent)
    left_mean / right_mean   per relation, freq / #distinct heads|tails  (bern, Reader.h:142-159)
    """

    def __init__(self, h, t, r, n_ent: int, n_rel: int):
        a = np.stack([np.asarray(h, np.int64), np.asarray(r, np.int64), np.asarray(t, np.int64)], 1)
        a = np.unique(a, axis=0)
        self.n_ent, self.n_rel = int(n_ent), int(n_rel)
        self.train_list = a
        self.head_hrt = a
        self.tail_hrt = a[np.lexsort((a[:, 0], a[:, 1], a[:, 2]))]
        self.rel_hrt = a[np.lexsort((a[:, 1], a[:, 2], a[:, 0]))]
        self.lef_head, self.rig_head = self._block(self.head_hrt[:, 0])
        self.lef_tail, self.rig_tail = self._block(self.tail_hrt[:, 2])
        self.lef_rel, self.rig_rel = self._block(self.rel_hrt[:, 0])
        freq = np.bincount(a[:, 1], minlength=n_rel).astype(np.float32)
        lcount = np.bincount(np.unique(a[:, :2], axis=0)[:, 1], minlength=n_rel).astype(np.float32)
        rcount = np.bincount(np.unique(a[:, [2, 1]], axis=0)[:, 1], minlength=n_rel).astype(np.float32)
        with np.errstate(divide="ignore", invalid="ignore"):
            self.left_mean = (freq / lcount).astype(np.float32)
            self.right_mean = (freq / rcount).astype(np.float32)

    def _block(self, keys):
        n = keys.shape[0]
        lef = np.zeros(self.n_ent, np.int64)
        rig = np.full(self.n_ent, -1, np.int64)
        first = np.ones(n, bool)
        first[1:] = keys[1:] != keys[:-1]
        last = np.ones(n, bool)
        last[:-1] = keys[1:] != keys[:-1]
        idx = np.arange(n)
        lef[keys[first]] = idx[first]
        rig[keys[last]] = idx[last]
        return lef, rig

    @property
    def train_total(self) -> int:
        return int(self.train_list.shape[0])
