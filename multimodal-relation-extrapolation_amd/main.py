"""Trainer-surface entry points of the reference's main.py that sit on the hot path.

evaluate(args, ent_embs, rel_embs, e2id, r2id, model, mode='test')  (main.py:217-272):
candidate ranking of every (head, relation) query of origin_data/<dataset>/<mode>/
<mode>_candidates.json ({relation: {"h\\tr\\t...": [true_tail, cand, ...]}}), scored with
NegativeSampling.evaluate (TransE L1, module/NegativeSampling.py:294-302) and ranked with
rank = #(s < p) + #(s == p) // 2 + 1 (main.py:245-250) -- all queries in one GPU launch
(csrc/candidates.hip) instead of a Python loop with per-candidate row copies. Prints the
per-relation and final lines of the reference and returns the final metrics.
The multimodal training loop of main.main (M3AE + RGCN) is upstream of the hot path."""
import json
import os
import os.path as osp

import numpy as np
import torch

from mmre.candidates import candidate_rank_transe


def build_candidates(test_candidates, e2id, r2id):
    qh, qr, off, ids, rel_names, rel_of_q = [], [], [0], [], [], []
    for query in test_candidates.keys():
        rel_names.append(query)
        for e1_rel, tails in test_candidates[query].items():
            head, rela, _ = e1_rel.split("\t")
            qh.append(e2id[head])
            qr.append(r2id[rela])
            ids.extend(e2id[t] for t in tails)
            off.append(len(ids))
            rel_of_q.append(len(rel_names) - 1)
    return (np.array(qh, np.int64), np.array(qr, np.int64), np.array(off, np.int64), np.array(ids, np.int64),
            rel_names, np.array(rel_of_q, np.int64))


def evaluate(args, ent_embs, rel_embs, e2id, r2id, model=None, mode="test", test_candidates=None, device=None):
    if test_candidates is None:
        data_path = osp.join("./origin_data", args.dataset)
        with open(os.path.join(data_path, f"{mode}/{mode}_candidates.json"), "r") as f:
            test_candidates = json.load(f)
    print("Start evaluation!\n")
    if model is not None:
        model.eval()
    dev = torch.device(device or "cuda:0")
    qh, qr, off, ids, rel_names, rel_of_q = build_candidates(test_candidates, e2id, r2id)
    to = lambda a: torch.as_tensor(a).to(dev)
    ent = torch.as_tensor(ent_embs, dtype=torch.float32).to(dev)
    rel = torch.as_tensor(rel_embs, dtype=torch.float32).to(dev)
    ranks = candidate_rank_transe(ent, rel, to(qh), to(qr), to(off), to(ids)).cpu().numpy().astype(np.int64)
    for i, query in enumerate(rel_names):
        tr = [int(x) for x in ranks[rel_of_q == i]]
        n = len(tr)
        print("Relation: %s| Number %d | mrr: %.4f | hit1: %.4f | hit3: %.4f | hit10: %.4f " % (
            query, len(test_candidates[query]), sum(1.0 / r for r in tr) / n,
            sum(1.0 if r <= 1 else 0.0 for r in tr) / n, sum(1.0 if r <= 3 else 0.0 for r in tr) / n,
            sum(1.0 if r <= 10 else 0.0 for r in tr) / n))
    rl = [int(x) for x in ranks]
    mrr = sum(1.0 / r for r in rl) / len(rl)
    hits = [sum(1.0 if r <= k else 0.0 for r in rl) / len(rl) for k in (1, 3, 10)]
    print(f"[Final Scores] MRR: {mrr} \tHits@1: {hits[0]} \tHits@3: {hits[1]} \tHits@10: {hits[2]}")
    return {"mrr": mrr, "hit1": hits[0], "hit3": hits[1], "hit10": hits[2], "ranks": ranks}
