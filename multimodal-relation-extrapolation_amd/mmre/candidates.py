"""Candidate-list rankings (csrc/candidates.hip): main.evaluate's TransE rank rule
(main.py:232-250) and ZSLmodule.eval's cosine rank (zsl_module.py:699-706)."""
from __future__ import annotations

import numpy as np
import torch

from ._lib import call, ptr, require_cuda, stream_ptr


def candidate_rank_transe(ent, rel, qh, qr, cand_off, cand_ids, return_scores=False):
    """ranks (Q,) int32 = #(s < p) + #(s == p) // 2 + 1, true candidate first in each list."""
    require_cuda(ent, rel, qh, qr, cand_off, cand_ids)
    n = int(qh.shape[0])
    dev = ent.device
    rank = torch.empty(n, dtype=torch.int32, device=dev)
    scores = torch.empty(int(cand_ids.shape[0]), dtype=torch.float32, device=dev) if return_scores else None
    call("mmre_candidate_rank_transe", ptr(ent.contiguous()), ptr(rel.contiguous()), int(ent.shape[1]),
         ptr(qh.contiguous()), ptr(qr.contiguous()), n, ptr(cand_off.contiguous()), ptr(cand_ids.contiguous()),
         ptr(scores), ptr(rank), stream_ptr(dev))
    return (rank, scores) if return_scores else rank


def cosine_rank(cand, cand_off, rel_vecs, rel_of_query, return_scores=False):
    """cand (C, d), rel_vecs (n_rel_sets, S, d) -> ranks (Q,) int32 of the first candidate."""
    require_cuda(cand, cand_off, rel_vecs, rel_of_query)
    n = int(rel_of_query.shape[0])
    dev = cand.device
    rank = torch.empty(n, dtype=torch.int32, device=dev)
    scores = torch.empty(int(cand.shape[0]), dtype=torch.float32, device=dev) if return_scores else None
    call("mmre_cosine_rank", ptr(cand.contiguous()), int(cand.shape[1]), ptr(cand_off.contiguous()), n,
         ptr(rel_vecs.contiguous()), int(rel_vecs.shape[1]), ptr(rel_of_query.contiguous()), ptr(scores), ptr(rank),
         stream_ptr(dev))
    return (rank, scores) if return_scores else rank


def hits_mrr(ranks, ks=(1, 3, 10)):
    """main.evaluate's final metrics (main.py:263-272) from integer ranks (python floats)."""
    r = [int(x) for x in np.asarray(ranks).tolist()]
    out = {"mrr": sum(1.0 / x for x in r) / len(r)}
    for k in ks:
        out[f"hit{k}"] = sum(1.0 if x <= k else 0.0 for x in r) / len(r)
    return out
