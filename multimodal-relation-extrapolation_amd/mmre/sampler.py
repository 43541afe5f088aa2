"""GPU negative samplers (csrc/sampler.hip).

OpenKESampler reproduces Base.so's `sampling` (Base.cpp:161-197) bit-for-bit, including the
per-thread LCG state carried across calls and the seeds randReset draws from the process's
glibc rand() stream (Random.h:11-15). RepoSampler is module/NegativeSampling.py's per-edge
filtered sampler (:114-140, :321-375) with a reproducible counter-based generator.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import call, lib, ptr, stream_ptr
from .data import TrainIndex


def glibc_seeds(n: int, skip: int = 0) -> np.ndarray:
    out = np.zeros(n, np.int64)
    call("mmre_glibc_rand", skip, n, out.ctypes.data_as(ctypes.c_void_p))
    return out.astype(np.uint64)


class OpenKESampler:
    def __init__(self, index: TrainIndex, device, work_threads: int = 8, bern: bool = False,
                 seeds: np.ndarray | None = None, seed_skip: int = 0, train_total: int | None = None):
        self.index = index
        self.device = torch.device(device)
        self.work_threads = int(work_threads)
        self.bern = bool(bern)
        self._seeds_dev = torch.empty(self.work_threads, dtype=torch.int64, device=self.device)
        self._ticket = torch.zeros(1, dtype=torch.int32, device=self.device)  # mmre_sampler_openke_step
        self.seeds = (np.asarray(seeds, np.uint64).copy() if seeds is not None
                      else glibc_seeds(self.work_threads, seed_skip))
        self.train_total = int(train_total if train_total is not None else index.train_total)
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        ix = index
        self._d = {k: to(getattr(ix, k)) for k in ("train_list", "head_hrt", "tail_hrt", "rel_hrt", "lef_head",
                                                   "rig_head", "lef_tail", "rig_tail", "lef_rel", "rig_rel",
                                                   "left_mean", "right_mean")}
        # each train row's (h, r) / (t, r) blocks, looked up once here instead of by two binary
        # searches per sampled negative (mmre_sampler_blocks)
        d = self._d
        self._n_blocks = int(ix.train_list.shape[0])
        self._blocks = torch.empty((self._n_blocks, 8), dtype=torch.int32, device=self.device)
        call("mmre_sampler_blocks", ptr(d["train_list"]), self._n_blocks, ptr(d["head_hrt"]), ptr(d["tail_hrt"]),
             ptr(d["lef_head"]), ptr(d["rig_head"]), ptr(d["lef_tail"]), ptr(d["rig_tail"]), ptr(self._blocks),
             stream_ptr(self.device))
        self.prob = None  # importProb's table (sample(..., p=True))
        self._prob_dev = None

    def import_prob(self, path: str, temperature: float):
        """importProb (Reader.h:26-49): the KL-weighted relation table sample(..., p=True) draws
        relation negatives from (Corrupt.h:111-147). path: the dataset's kl_prob.txt (n_rel x
        (n_rel - 1) floats), read and weighted by mmre_import_prob exactly as the reference."""
        R = self.index.n_rel
        prob = np.zeros((R, R - 1), np.float32)
        call("mmre_import_prob", str(path).encode(), R, float(temperature), prob.ctypes.data_as(ctypes.c_void_p))
        self.prob = prob
        self._prob_dev = torch.from_numpy(prob).to(self.device)
        return prob

    @property
    def seeds(self) -> np.ndarray:
        """The per-pthread LCG states (Random.h next_random[]), host mirror of the device copy."""
        return self._seeds

    @seeds.setter
    def seeds(self, value):
        self._seeds = np.asarray(value, np.uint64).copy()
        self._seeds_dev.copy_(torch.from_numpy(self._seeds.view(np.int64)))
        self.draws = getattr(self, "draws", 0) + 1

    # draws: bumped by every batch drawn and every seed reset -- a prefetching consumer
    # (mmre.ns.OpenKETrainStep) checks that nobody else drew from this sampler since its prefetch

    def sample(self, batch_size: int, neg_ent: int = 1, neg_rel: int = 0, mode: int = 0, out=None, p: bool = False):
        """Base.cpp:161-197 sampling(batch, neg_ent, neg_rel, mode, filter_flag, p); p=True draws the
        relation negatives from import_prob's table (Corrupt.h:111-147)."""
        B = int(batch_size)
        n = B * (1 + neg_ent + neg_rel)
        dev = self.device
        if out is None:
            out = dict(batch_h=torch.empty(n, dtype=torch.int64, device=dev),
                       batch_t=torch.empty(n, dtype=torch.int64, device=dev),
                       batch_r=torch.empty(n, dtype=torch.int64, device=dev),
                       batch_y=torch.empty(n, dtype=torch.float32, device=dev))
        d = self._d
        # one launch: the batch, and the per-thread LCG states advanced (by a fixed number of draws
        # per positive) for the next call by the kernel's last workgroup -- no host copy per batch
        use_p = bool(p) and int(neg_rel) > 0
        if use_p and self._prob_dev is None:
            raise ValueError("sample(p=True) needs import_prob() first (Reader.h:26)")
        args = (ptr(d["train_list"]), self.train_total, ptr(d["head_hrt"]),
                ptr(d["tail_hrt"]), ptr(d["rel_hrt"]), ptr(d["lef_head"]), ptr(d["rig_head"]), ptr(d["lef_tail"]),
                ptr(d["rig_tail"]), ptr(d["lef_rel"]), ptr(d["rig_rel"]), ptr(d["left_mean"]) if self.bern else None,
                ptr(d["right_mean"]) if self.bern else None, self.index.n_ent, self.index.n_rel,
                ptr(self._seeds_dev), self.work_threads, B, int(neg_ent), int(neg_rel), int(mode),
                ptr(self._blocks), self._n_blocks, ptr(out["batch_h"]), ptr(out["batch_t"]), ptr(out["batch_r"]),
                ptr(out["batch_y"]), ptr(self._ticket))
        if use_p:
            call("mmre_sampler_openke_p", *args, ptr(self._prob_dev), stream_ptr(dev))
        else:
            call("mmre_sampler_openke_step", *args, stream_ptr(dev))
        # ... and the host mirror
        call("mmre_sampler_advance", self._seeds.ctypes.data_as(ctypes.c_void_p), self.work_threads, B,
             int(neg_ent), int(neg_rel), int(mode))
        self.draws += 1
        return out


    def advance(self, batch_size: int, neg_ent: int, mode: int):
        """Advance the host mirror by one batch a kernel drew (the device seeds advance there)."""
        call("mmre_sampler_advance", self._seeds.ctypes.data_as(ctypes.c_void_p), self.work_threads, int(batch_size),
             int(neg_ent), 0, int(mode))
        self.draws += 1

    def step_args(self, batch_size: int, neg_ent: int, mode: int, out, advance: bool = True):
        """The sampler half of mmre_ns_step_openke's arguments (the step's launch samples the batch
        into `out` and advances the device seeds); the host mirror advances here, as sample() does
        (advance=False: the arguments only -- the batch was drawn by an earlier launch)."""
        d = self._d
        args = (ptr(d["train_list"]), self.train_total, ptr(d["head_hrt"]), ptr(d["tail_hrt"]), ptr(d["rel_hrt"]),
                ptr(d["lef_head"]), ptr(d["rig_head"]), ptr(d["lef_tail"]), ptr(d["rig_tail"]), ptr(d["lef_rel"]),
                ptr(d["rig_rel"]), ptr(d["left_mean"]) if self.bern else None,
                ptr(d["right_mean"]) if self.bern else None, ptr(self._seeds_dev), self.work_threads, int(mode),
                ptr(self._blocks), self._n_blocks, ptr(out["batch_h"]), ptr(out["batch_t"]), ptr(out["batch_r"]),
                ptr(out["batch_y"]), ptr(self._ticket))
        if advance:
            self.advance(batch_size, neg_ent, mode)
        return args


class RepoSampler:
    """module/NegativeSampling.py's filtered per-edge sampler on the GPU.

    whole_triples: ([h], [r], [t]) global ids (NegativeSampling.py:56-58 __count_htr)."""

    def __init__(self, whole_triples, n_rel: int, device, filter_flag: bool = True, seed: int = 0):
        h, r, t = (np.asarray(x, np.int64) for x in whole_triples)
        self.n_rel = int(n_rel)
        self.device = torch.device(device)
        self.filter_flag = bool(filter_flag)
        self.seed = int(seed)
        self.calls = 0
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        # heads of (t, r): key t * R + r ; tails of (h, r): key h * R + r
        self.hf = [to(x) for x in self._csr(t * self.n_rel + r, h)]
        self.tf = [to(x) for x in self._csr(h * self.n_rel + r, t)]

    @staticmethod
    def _csr(keys, vals):
        kv = np.unique(np.stack([keys, vals], 1), axis=0)
        uk, start = np.unique(kv[:, 0], return_index=True)
        off = np.append(start, len(kv)).astype(np.int64)
        return uk.astype(np.int64), off, kv[:, 1].astype(np.int64)

    def sample(self, edge_index: torch.Tensor, edge_type: torch.Tensor, neg_ent: int, n_local: int,
               local_to_global: torch.Tensor | None = None):
        """edge_index (2, B) local ids, edge_type (B,) -> expanded (2, B(1+k)), (B(1+k),) int64
        in the layout [pos | neg_1 | ... | neg_k] (NegativeSampling.py:121-139)."""
        dev = self.device
        B = int(edge_type.shape[0])
        eh = edge_index[0].to(dev, torch.int64).contiguous()
        et = edge_index[1].to(dev, torch.int64).contiguous()
        er = edge_type.to(dev, torch.int64).contiguous()
        n = B * (1 + int(neg_ent))
        oh = torch.empty(n, dtype=torch.int64, device=dev)
        ot = torch.empty(n, dtype=torch.int64, device=dev)
        orr = torch.empty(n, dtype=torch.int64, device=dev)
        l2g = None if local_to_global is None else local_to_global.to(dev, torch.int64).contiguous()
        hk, ho, hv = self.hf
        tk, to_, tv = self.tf
        call("mmre_sampler_repo", ptr(eh), ptr(et), ptr(er), B, int(neg_ent), int(n_local), ptr(l2g), self.n_rel,
             ptr(hk), ptr(ho), ptr(hv), int(hk.shape[0]), ptr(tk), ptr(to_), ptr(tv), int(tk.shape[0]),
             ctypes.c_uint64((self.seed * 0x9E3779B97F4A7C15 + self.calls) & 0xFFFFFFFFFFFFFFFF),
             int(self.filter_flag), ptr(oh), ptr(ot), ptr(orr), stream_ptr(dev))
        self.calls += 1
        return torch.stack([oh, ot]), orr
