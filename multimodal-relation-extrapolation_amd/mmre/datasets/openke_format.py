"""OpenKE-format dataset files: the on-disk input of the link-prediction path.

Base.so's readers (Reader.h:53-317) and this package's loaders (mmre.data.OpenKEDataset,
libmmre_base.so) consume a directory of:

    entity2id.txt / relation2id.txt   count, then "name<TAB>id" lines   (OpenKE/README.md:126-141)
    train2id.txt / valid2id.txt / test2id.txt   count, then "h t r" lines
    type_constrain.txt                allowed heads / tails per relation (Reader.h:266-317)
    1-1.txt 1-n.txt n-1.txt n-n.txt test2id_all.txt   test triples by relation category

`postprocess(dir)` produces the last group from the three triple files with the rules of the
reference's post-processing script (utils/n-n.py, OpenKE/benchmarks/*/n-n.py): relations and
entities listed in first-appearance order over train, valid, test; a relation is "1-n" etc. by
its mean tails per (h, r) and heads per (r, t) against 1.5. On the reference's shipped
OpenKE/benchmarks/FB15K237 inputs the category files come out byte-identical to the shipped
ones and type_constrain.txt has identical per-relation head/tail sets (the shipped file's line
order is an old Python's dict order; Reader.h is order-independent) -- tests/test_openke_format.py.

`from_zs(origin_dir, out_dir)` converts the repo's zero-shot datasets (origin_data/<name>:
entity2ids_zsl.json, relation2ids.json, test_tasks_zsl.json, read as zsl_module.py:146-151
does) into that format, so the OpenKE Tester path and Base.so-compatible library can evaluate
them.
"""
from __future__ import annotations

import json
import os

import numpy as np

CATEGORY_FILES = ("1-1.txt", "1-n.txt", "n-1.txt", "n-n.txt")


def _read_lines(path):
    """(count, raw lines) of an OpenKE triple file; the count line decides how many are used."""
    with open(path) as f:
        n = int(f.readline())
        return [f.readline() for _ in range(n)]


def write_ids(path, names_by_id):
    with open(path, "w") as f:
        f.write(f"{len(names_by_id)}\n")
        for i, name in enumerate(names_by_id):
            f.write(f"{name}\t{i}\n")


def write_triples(path, h, t, r):
    h, t, r = (np.asarray(x, np.int64) for x in (h, t, r))
    with open(path, "w") as f:
        f.write(f"{len(h)}\n")
        f.writelines(f"{a} {b} {c}\n" for a, b, c in zip(h.tolist(), t.tolist(), r.tolist()))


def postprocess(directory):
    """Write type_constrain.txt and the relation-category test splits of an OpenKE directory."""
    path = lambda name: os.path.join(directory, name)
    heads_of, tails_of = {}, {}      # relation -> {entity: None}, first-appearance order
    per_hr, per_rt = {}, {}          # (h, r) -> #tails listed, (r, t) -> #heads listed
    for name in ("train2id.txt", "valid2id.txt", "test2id.txt"):
        for line in _read_lines(path(name)):
            h, t, r = line.strip().split()
            per_hr[(h, r)] = per_hr.get((h, r), 0) + 1
            per_rt[(r, t)] = per_rt.get((r, t), 0) + 1
            heads_of.setdefault(r, {})[h] = None
            tails_of.setdefault(r, {})[t] = None
    with open(path("type_constrain.txt"), "w") as f:
        f.write(f"{len(heads_of)}\n")
        for r, hs in heads_of.items():
            f.write(f"{r}\t{len(hs)}" + "".join(f"\t{e}" for e in hs) + "\n")
            ts = tails_of[r]
            f.write(f"{r}\t{len(ts)}" + "".join(f"\t{e}" for e in ts) + "\n")
    # mean tails per (h, r) key and heads per (r, t) key, per relation
    tail_sum, hr_keys, head_sum, rt_keys = {}, {}, {}, {}
    for (h, r), n in per_hr.items():
        tail_sum[r] = tail_sum.get(r, 0) + n
        hr_keys[r] = hr_keys.get(r, 0.0) + 1.0
    for (r, t), n in per_rt.items():
        head_sum[r] = head_sum.get(r, 0) + n
        rt_keys[r] = rt_keys.get(r, 0.0) + 1.0
    test = _read_lines(path("test2id.txt"))
    cats = []
    for line in test:
        h, t, r = line.strip().split()
        many_tails = tail_sum[r] / hr_keys[r] >= 1.5
        many_heads = head_sum[r] / rt_keys[r] >= 1.5
        cats.append(int(many_tails) + 2 * int(many_heads))   # 0 1-1, 1 1-n, 2 n-1, 3 n-n
    for c, name in enumerate(CATEGORY_FILES):
        lines = [l for l, k in zip(test, cats) if k == c]
        with open(path(name), "w") as f:
            f.write(f"{len(lines)}\n")
            f.writelines(lines)
    with open(path("test2id_all.txt"), "w") as f:
        f.write(f"{len(test)}\n")
        f.writelines(f"{k}\t{l}" for l, k in zip(test, cats))


def read_zs(origin_dir):
    """Entity / relation names by id and the test triples (h, t, r ids, task-file order) of a
    zero-shot dataset directory. Triples whose names are missing from the id maps are dropped
    (counted in `unmapped`)."""
    load = lambda name: json.load(open(os.path.join(origin_dir, name)))
    e2id, r2id, tasks = load("entity2ids_zsl.json"), load("relation2ids.json"), load("test_tasks_zsl.json")
    ents = [None] * len(e2id)
    for name, i in e2id.items():
        ents[i] = name
    rels = [None] * len(r2id)
    for name, i in r2id.items():
        rels[i] = name
    h, t, r, unmapped = [], [], [], 0
    for triples in tasks.values():
        for a, b, c in triples:
            if a in e2id and c in e2id and b in r2id:
                h.append(e2id[a]); t.append(e2id[c]); r.append(r2id[b])
            else:
                unmapped += 1
    return dict(entities=ents, relations=rels, h=np.array(h, np.int64), t=np.array(t, np.int64),
                r=np.array(r, np.int64), unmapped=unmapped)


def from_zs(origin_dir, out_dir, train=None, valid=None):
    """Write an OpenKE directory for a zero-shot dataset. train / valid: optional (h, t, r) id
    arrays (the repo's train_tasks_zsl.json is not shipped); absent -> empty files."""
    z = read_zs(origin_dir)
    os.makedirs(out_dir, exist_ok=True)
    write_ids(os.path.join(out_dir, "entity2id.txt"), z["entities"])
    write_ids(os.path.join(out_dir, "relation2id.txt"), z["relations"])
    write_triples(os.path.join(out_dir, "test2id.txt"), z["h"], z["t"], z["r"])
    empty = (np.zeros(0, np.int64),) * 3
    write_triples(os.path.join(out_dir, "train2id.txt"), *(train if train is not None else empty))
    write_triples(os.path.join(out_dir, "valid2id.txt"), *(valid if valid is not None else empty))
    postprocess(out_dir)
    return z
