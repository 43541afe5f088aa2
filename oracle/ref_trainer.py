"""ref_trainer.py -- TEST INFRASTRUCTURE ONLY: the reference's CPU training step for the
negative-sampling path, as bench.py's `cpu_baseline` leg of --config ns and as the float
reference of the fused loss in the GPU parity tests.

One OpenKE training step (Trainer.train_one_step, OpenKE/openke/config/Trainer.py:43-54):

    Base.so sampling (Base.cpp:161-197, the reference's own C++: oracle/_ref, pthreads)
    -> TransE.forward in 'normal' mode (TransE.py:46-74) on torch CPU
    -> strategy NegativeSampling.forward (strategy/NegativeSampling.py:13-32):
       _get_positive_score / _get_negative_score -> MarginLoss (MarginLoss.py:24-28)
       (+ regul_rate * regularization, TransE.py:76-86)
    -> loss.backward() -> SGD step.

`transe_ns_loss` is that op sequence over explicit tables (no nn.Module), so the GPU tests can
evaluate it in float64 on the GPU sampler's batch. Usage as a child of bench.py:
    python oracle/ref_trainer.py <workdir>
<workdir> holds the OpenKE files (entity2id / relation2id / train2id) and meta.json (dim,
batch, neg, margin, norm_flag, bern, steps, threads); the result goes to <workdir>/result.json.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_BASE_SO = os.path.join(HERE, "_ref", "Base.so")


def transe_ns_loss(ent, rel, h, t, r, batch_size, margin, norm_flag=True, p_norm=1, adv_temperature=None,
                   regul_rate=0.0):
    """strategy NegativeSampling.forward over TransE (normal mode) + MarginLoss, torch ops in
    the reference's order; differentiable w.r.t. ent / rel (any dtype)."""
    import torch
    import torch.nn.functional as F
    hv, tv, rv = ent[h], ent[t], rel[r]
    hn, tn, rn = hv, tv, rv
    if norm_flag:
        hn = F.normalize(hv, 2, -1)
        rn = F.normalize(rv, 2, -1)
        tn = F.normalize(tv, 2, -1)
    score = torch.norm((hn + rn) - tn, p_norm, -1).flatten()            # TransE._calc, mode 'normal'
    p = score[:batch_size].view(-1, batch_size).permute(1, 0)
    n = score[batch_size:].view(-1, batch_size).permute(1, 0)
    m = torch.tensor([margin], dtype=ent.dtype)
    if adv_temperature is not None:
        w = F.softmax(-n * adv_temperature, dim=-1).detach()
        loss = (w * torch.max(p - n, -m)).sum(dim=-1).mean() + m
    else:
        loss = torch.max(p - n, -m).mean() + m
    if regul_rate != 0:
        loss = loss + regul_rate * (torch.mean(hv ** 2) + torch.mean(tv ** 2) + torch.mean(rv ** 2)) / 3
    return loss[0] if loss.dim() else loss, score


def model_ns_loss(model, tables, h, t, r, batch_size, margin, adv_temperature=None, regul_rate=0.0,
                  model_margin=6.0, epsilon=2.0):
    """strategy NegativeSampling.forward (strategy/NegativeSampling.py:13-32) over DistMult /
    ComplEx / RotatE in 'normal' mode + MarginLoss (+ regularization), the reference's op
    sequences (DistMult.py:34-66, ComplEx.py:20-55, RotatE.py:45-103) over explicit tables
    {ent, rel[, ent_im, rel_im]}; differentiable w.r.t. them (any dtype)."""
    import math

    import torch
    import torch.nn.functional as F
    if model == "distmult":
        hv, tv, rv = tables["ent"][h], tables["ent"][t], tables["rel"][r]
        score = torch.sum((hv * rv) * tv, -1).flatten()
        regs = [hv, tv, rv]
    elif model == "complex":
        er, ei, rr_, ri = tables["ent"], tables["ent_im"], tables["rel"], tables["rel_im"]
        h_re, h_im, t_re, t_im, r_re, r_im = er[h], ei[h], er[t], ei[t], rr_[r], ri[r]
        score = torch.sum(h_re * t_re * r_re + h_im * t_im * r_re + h_re * t_im * r_im - h_im * t_re * r_im, -1)
        regs = [h_re, h_im, t_re, t_im, r_re, r_im]
    elif model == "rotate":
        hv, tv, rv = tables["ent"][h], tables["ent"][t], tables["rel"][r]
        dim = rv.shape[-1]
        rng = torch.tensor([(model_margin + epsilon) / dim], dtype=torch.float32).to(rv.dtype)
        re_h, im_h = torch.chunk(hv, 2, dim=-1)
        re_t, im_t = torch.chunk(tv, 2, dim=-1)
        phase = rv / (rng.item() / math.pi)
        re_r, im_r = torch.cos(phase), torch.sin(phase)
        re_s = re_h * re_r - im_h * im_r - re_t
        im_s = re_h * im_r + im_h * re_r - im_t
        score = model_margin - torch.stack([re_s, im_s], dim=0).norm(dim=0).sum(dim=-1).flatten()
        regs = [hv, tv, rv]
    else:
        raise ValueError(model)
    p = score[:batch_size].view(-1, batch_size).permute(1, 0)
    n = score[batch_size:].view(-1, batch_size).permute(1, 0)
    m = torch.tensor([margin], dtype=score.dtype)
    if adv_temperature is not None:
        w = F.softmax(-n * adv_temperature, dim=-1).detach()
        loss = (w * torch.max(p - n, -m)).sum(dim=-1).mean() + m
    else:
        loss = torch.max(p - n, -m).mean() + m
    if regul_rate != 0:
        loss = loss + regul_rate * sum(torch.mean(x ** 2) for x in regs) / len(regs)
    return loss[0] if loss.dim() else loss, score


def run_trainer(workdir: str, base_so: str = REF_BASE_SO):
    import torch
    with open(os.path.join(workdir, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("threads"):
        torch.set_num_threads(int(meta["threads"]))
    lib = ctypes.CDLL(base_so)
    P, I = ctypes.c_void_p, ctypes.c_int64
    lib.setInPath.argtypes = [ctypes.c_char_p]
    lib.setBern.argtypes = [I]
    lib.setWorkThreads.argtypes = [I]
    lib.sampling.argtypes = [P, P, P, P, I, I, I, I, ctypes.c_bool, ctypes.c_bool, ctypes.c_bool]
    lib.getEntityTotal.restype = I
    lib.getRelationTotal.restype = I
    saved = os.dup(1)
    os.dup2(2, 1)  # Base.so printf()s to fd 1
    try:
        lib.setInPath((workdir.rstrip("/") + "/").encode())
        lib.setBern(int(bool(meta.get("bern", True))))
        lib.setWorkThreads(int(meta.get("sampler_threads", 8)))
        lib.randReset()
        lib.importTrainFiles()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    E, R = int(lib.getEntityTotal()), int(lib.getRelationTotal())
    d, B, k = int(meta["dim"]), int(meta["batch"]), int(meta["neg"])
    n = B * (1 + k)
    g = torch.Generator().manual_seed(0)
    bound_e, bound_r = (6.0 / (E + d)) ** 0.5, (6.0 / (R + d)) ** 0.5   # xavier_uniform_ (TransE.py:20-22)
    ent = ((torch.rand((E, d), generator=g) * 2 - 1) * bound_e).requires_grad_(True)
    rel = ((torch.rand((R, d), generator=g) * 2 - 1) * bound_r).requires_grad_(True)
    opt = torch.optim.SGD([ent, rel], lr=float(meta.get("lr", 1.0)))
    bh, bt, br = (np.zeros(n, np.int64) for _ in range(3))
    by = np.zeros(n, np.float32)
    steps = int(meta["steps"])
    times = {"sampling": 0.0, "forward": 0.0, "backward_step": 0.0}
    loss = None
    t_all = time.perf_counter()
    for _ in range(steps):
        t0 = time.perf_counter()
        lib.sampling(bh.ctypes.data, bt.ctypes.data, br.ctypes.data, by.ctypes.data, B, k, 0, 0, True, False, False)
        t1 = time.perf_counter()
        opt.zero_grad()
        loss, _ = transe_ns_loss(ent, rel, torch.from_numpy(bh), torch.from_numpy(bt), torch.from_numpy(br), B,
                                 float(meta["margin"]), norm_flag=bool(meta.get("norm_flag", True)))
        t2 = time.perf_counter()
        loss.backward()
        opt.step()
        t3 = time.perf_counter()
        times["sampling"] += t1 - t0
        times["forward"] += t2 - t1
        times["backward_step"] += t3 - t2
    elapsed = time.perf_counter() - t_all
    out = dict(elapsed=elapsed, steps=steps, threads=torch.get_num_threads(), rows_per_step=n,
               times=times, final_loss=float(loss.detach()) if loss is not None else None, n_ent=E, n_rel=R)
    with open(os.path.join(workdir, "result.json"), "w") as f:
        json.dump(out, f)
    return out


if __name__ == "__main__":
    r = run_trainer(sys.argv[1])
    print(f"ref_trainer: {r['steps']} steps in {r['elapsed']:.2f} s on {r['threads']} threads")
