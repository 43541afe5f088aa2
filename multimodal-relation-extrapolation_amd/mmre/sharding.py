"""Relation-sharded multi-GPU evaluation.

Whole test relations are assigned to ranks by LPT packing of their query counts, so every
rank keeps Test.h's relation-major order (testList sorted by (r, h, t), Reader.h:227) for its
queries and reuses its relations' rows. Entity and relation tables are replicated (11-60 MB at
the ZS configs, far below 288 GB). After the local sweep, ONE all-gather of the per-rank int32
rank-count lists (RCCL over xGMI; gloo on CPU in tests) lets every rank reduce the metrics in
the reference's sequential order, so rank 0's metrics are bit-equal to the single-GPU run.
"""
from __future__ import annotations

import numpy as np
import torch


def lpt_partition(rel_of_query: np.ndarray, world: int):
    """Assign relations to `world` ranks, heaviest first onto the least-loaded rank.
    Returns a list of boolean masks over queries (one per rank)."""
    rel_of_query = np.asarray(rel_of_query)
    rels, counts = np.unique(rel_of_query, return_counts=True)
    order = np.lexsort((rels, -counts))  # heaviest first, ties by relation id (deterministic)
    load = np.zeros(world, np.int64)
    owner = {}
    for i in order:
        k = int(np.argmin(load))
        owner[int(rels[i])] = k
        load[k] += counts[i]
    own = np.array([owner[int(r)] for r in rel_of_query]) if len(rel_of_query) else np.zeros(0, int)
    return [own == k for k in range(world)]


class ShardPlan:
    """Everything each rank precomputes once from the (deterministic, identical on every rank)
    lpt_partition masks: its own query ids, the padded width, and the device index maps that
    put all-gathered columns back into global query order."""

    def __init__(self, masks, device):
        self.world = len(masks)
        self.n_total = len(masks[0])
        self.sizes = [int(m.sum()) for m in masks]
        self.pad = max(max(self.sizes), 1)
        self.ids = [np.nonzero(m)[0] for m in masks]
        cols, dst = [], []
        for k in range(self.world):
            cols.append(k * self.pad + np.arange(self.sizes[k]))
            dst.append(self.ids[k])
        self.cols = torch.from_numpy(np.concatenate(cols).astype(np.int64)).to(device)
        self.dst = torch.from_numpy(np.concatenate(dst).astype(np.int64)).to(device)
        self.device = device


def gather_counts(local_counts: torch.Tensor, plan: ShardPlan, group=None):
    """All-gather per-rank (4, n_local) int32 count lists into global query order: ONE
    collective of world x 4 x pad int32 (about 282 KB in total at FB15K-237-ZS), no index
    exchange (every rank knows the partition)."""
    import torch.distributed as dist
    buf = torch.zeros((4, plan.pad), dtype=torch.int32, device=plan.device)
    buf[:, :local_counts.shape[1]] = local_counts
    out = torch.empty((plan.world, 4, plan.pad), dtype=torch.int32, device=plan.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    full = torch.empty((4, plan.n_total), dtype=torch.int32, device=plan.device)
    full[:, plan.dst] = out.permute(1, 0, 2).reshape(4, -1)[:, plan.cols]
    return full
