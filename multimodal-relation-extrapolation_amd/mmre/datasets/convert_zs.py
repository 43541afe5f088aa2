"""Build mmre/datasets/*_test.npz from the reference's zero-shot datasets.

Runs in the build container only (reads /root/reference/origin_data, which does not exist on
the GPU box); the .npz files it writes are committed. They hold only integer ids:
test_tasks_zsl.json triples mapped through entity2ids_zsl.json and relation2ids.json, in the
file's relation order (as ZSLmodule / main.evaluate read them, zsl_module.py:146-151).
"""
import json
import os
import sys

import numpy as np

SRC = "/root/reference/origin_data"
OUT = os.path.dirname(os.path.abspath(__file__))


def convert(name, out):
    d = os.path.join(SRC, name)
    e2id = json.load(open(os.path.join(d, "entity2ids_zsl.json")))
    r2id = json.load(open(os.path.join(d, "relation2ids.json")))
    tasks = json.load(open(os.path.join(d, "test_tasks_zsl.json")))
    h, r, t = [], [], []
    missing = 0
    for rel, triples in tasks.items():
        for (a, b, c) in triples:
            if a not in e2id or c not in e2id or b not in r2id:
                missing += 1
                continue
            h.append(e2id[a]); r.append(r2id[b]); t.append(e2id[c])
    np.savez_compressed(os.path.join(OUT, out), h=np.array(h, np.int32), r=np.array(r, np.int32),
                        t=np.array(t, np.int32), n_ent=np.array(len(e2id)), n_rel=np.array(len(r2id)),
                        missing=np.array(missing))
    print(name, "triples", len(h), "E", len(e2id), "R", len(r2id), "unmapped", missing,
          "relations", len(set(r)))


def convert_candidates(name, out):
    """rel2candidates_all.json (the candidate pool gen_mode_candidates.py filters per test
    triple, utils/gen_mode_candidates.py:27-34) for the test relations, as entity ids in the
    order of test_tasks_zsl.json's relations (rel_ids) -- (n_test_rel, n_cand) with -1 for names
    absent from entity2ids_zsl.json."""
    d = os.path.join(SRC, name)
    e2id = json.load(open(os.path.join(d, "entity2ids_zsl.json")))
    r2id = json.load(open(os.path.join(d, "relation2ids.json")))
    tasks = json.load(open(os.path.join(d, "test_tasks_zsl.json")))
    cands = json.load(open(os.path.join(d, "rel2candidates_all.json")))
    rels = list(tasks.keys())
    width = max(len(cands[r]) for r in rels)
    ids = np.full((len(rels), width), -1, np.int32)
    for i, r in enumerate(rels):
        for j, e in enumerate(cands[r]):
            ids[i, j] = e2id.get(e, -1)
    np.savez_compressed(os.path.join(OUT, out), rel_ids=np.array([r2id[r] for r in rels], np.int32), cand=ids)
    print(name, "candidate pools", ids.shape, "unmapped", int((ids < 0).sum()))


def convert_descriptions(name, out, max_len=320, vocab=30522, first_id=1000):
    """rel_description_zsl (one description per relation id, the rel_des_file that
    MMKGDataset.generate_batch indexes by relation, module/data.py:274, 301-304) as synthetic
    token rows: the BERT tokenizer (module/data.py:256-263, add_special_tokens=False,
    padding='max_length', truncation at unpaired_tokenizer_max_length = 320) is not available
    offline, so each description is split the way BERT's basic tokenizer splits (lower case,
    words and single punctuation marks) and every piece gets a stable id in [first_id, vocab).
    Lengths are therefore the pre-token counts (WordPiece can only add pieces). Writes tok
    (R, max_len) int32 with 0 on padded positions and n_tok (R,) int32."""
    import re
    import zlib
    d = os.path.join(SRC, name)
    lines = open(os.path.join(d, "rel_description_zsl")).read().splitlines()
    tok = np.zeros((len(lines), max_len), np.int32)
    n_tok = np.zeros(len(lines), np.int32)
    for i, line in enumerate(lines):
        pieces = re.findall(r"\w+|[^\w\s]", line.lower())[:max_len]
        ids = [first_id + zlib.crc32(p.encode()) % (vocab - first_id) for p in pieces]
        tok[i, :len(ids)] = ids
        n_tok[i] = len(ids)
    np.savez_compressed(os.path.join(OUT, out), tok=tok, n_tok=n_tok, vocab=np.array(vocab))
    print(name, "descriptions", len(lines), "tokens min/mean/max", n_tok.min(), round(float(n_tok.mean()), 1),
          n_tok.max())


if __name__ == "__main__":
    if not os.path.isdir(SRC):
        sys.exit("reference data not available")
    convert("FB15K-237-ZS", "fb15k237zs_test.npz")
    convert("DB15K-ZS", "db15kzs_test.npz")
    convert_candidates("FB15K-237-ZS", "fb15k237zs_cands.npz")
    convert_descriptions("FB15K-237-ZS", "fb15k237zs_desc.npz")
