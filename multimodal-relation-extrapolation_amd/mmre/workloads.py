"""Synthetic workloads of BASELINE.json's configs.

Real id spaces and test triples of the zero-shot datasets; OpenKE's own initialisation for
the tables (xavier_uniform_, TransE.py:36-38; RotatE's uniform range, RotatE.py:20-40) with
seed 0; the filter set is the test triples plus a synthetic "train" of uniformly random
triples sized like OpenKE FB15K237 (272,115), because train_tasks_zsl.json is not shipped.
"""
from __future__ import annotations

import numpy as np
import torch

from .data import load_zs_test, sorted_rel2

FB15K237_TRAIN = 272_115


def xavier(rows, cols, gen):
    bound = float(np.sqrt(6.0 / (rows + cols)))
    return (torch.rand((rows, cols), generator=gen, dtype=torch.float32) * 2 - 1) * bound


def zs_workload(dataset: str = "FB15K-237-ZS", model: str = "transe", dim: int = 200, seed: int = 0,
                margin: float = 6.0, epsilon: float = 2.0, n_train: int = FB15K237_TRAIN):
    z = load_zs_test(dataset)
    E, R = int(z["n_ent"]), int(z["n_rel"])
    gen = torch.Generator().manual_seed(seed)
    w = dict(dataset=dataset, model=model, dim=dim, n_ent=E, n_rel=R)
    if model in ("transe", "transe_l2", "distmult"):
        w["ent"], w["rel"] = xavier(E, dim, gen), xavier(R, dim, gen)
    elif model == "complex":
        w["ent"], w["ent_im"] = xavier(E, dim, gen), xavier(E, dim, gen)
        w["rel"], w["rel_im"] = xavier(R, dim, gen), xavier(R, dim, gen)
    elif model == "rotate":
        er = (margin + epsilon) / (2 * dim)
        rr = (margin + epsilon) / dim
        w["ent"] = (torch.rand((E, 2 * dim), generator=gen) * 2 - 1) * er
        w["rel"] = (torch.rand((R, dim), generator=gen) * 2 - 1) * rr
        w["margin"], w["epsilon"] = margin, epsilon
    # test triples in Test.h order (r, h, t)
    file_order = np.stack([z["h"], z["t"], z["r"]], 1).astype(np.int64)
    h, r, t = sorted_rel2(file_order)
    w["test_h"], w["test_r"], w["test_t"] = h, r, t
    rng = np.random.default_rng(seed + 2)
    th = rng.integers(0, E, n_train)
    tr = rng.integers(0, R, n_train)
    tt = rng.integers(0, E, n_train)
    w["filter_h"] = np.concatenate([th, h])
    w["filter_r"] = np.concatenate([tr, r])
    w["filter_t"] = np.concatenate([tt, t])
    return w


def synthetic_large(n_ent=1_000_000, n_rel=235, dim=256, n_query=8192, seed=0):
    """C5: synthetic |E| = 1M DistMult d=256 with 8,192 random queries."""
    gen = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed + 1)
    w = dict(dataset="synthetic-1M", model="distmult", dim=dim, n_ent=n_ent, n_rel=n_rel,
             ent=xavier(n_ent, dim, gen), rel=xavier(n_rel, dim, gen))
    w["test_h"] = rng.integers(0, n_ent, n_query // 2)
    w["test_r"] = rng.integers(0, n_rel, n_query // 2)
    w["test_t"] = rng.integers(0, n_ent, n_query // 2)
    w["filter_h"], w["filter_r"], w["filter_t"] = w["test_h"], w["test_r"], w["test_t"]
    return w
