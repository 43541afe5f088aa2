#!/usr/bin/env python
"""bench.py -- scored triples/s of the link-prediction sweep (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

One step = one complete filtered link-prediction evaluation of the configured workload
(default C2: FB15K-237-ZS test set, TransE d=200, norm_flag, all 17,596 test triples in both
head_batch and tail_batch mode = 35,192 sweeps over 14,208 entities): entity-table prep, query
vectors, truth scores + filter correction, the fused sweep + rank epilogue, (N>1) the RCCL
all-gather of per-rank rank-count lists, the D2H copy of the counts and the Test.h metric
reduction. Inputs (tables, queries, filter lists) are resident in HBM before timing starts.
N>1: launched by torch.distributed.run, one rank per GPU, relation-sharded (LPT) queries.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "multimodal-relation-extrapolation_amd")
for p in (PKG, REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "scored triples/sec + hit@10 parity, FB15K-237-ZS TransE d=200 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9   # 256 CUs x 4 SIMD-32 x 2.4 GHz (lane-ops/s)

CONFIGS = {
    "c1": dict(dataset="FB15K-237-ZS", model="transe", dim=100, norm=True, n_test=1000,
               workload="C1 FB15K-237-ZS TransE d=100 p=1 norm_flag, filtered link prediction of the first 1,000 "
                        "test triples (Test.h order)"),
    "c2": dict(dataset="FB15K-237-ZS", model="transe", dim=200, norm=True,
               workload="C2 FB15K-237-ZS TransE d=200 p=1 norm_flag, filtered link prediction"),
    "c3": dict(dataset="DB15K-ZS", model="complex", dim=200, norm=False,
               workload="C3 DB15K-ZS ComplEx d=200, filtered link prediction (split-bf16 MFMA filter, "
                        "exact f32 ranks)"),
    "c4": dict(dataset="FB15K-237-ZS", model="rotate", dim=512, norm=False,
               workload="C4 FB15K-237-ZS RotatE d=512, filtered link prediction"),
    "c5": dict(dataset="synthetic-1M", model="distmult", dim=256, norm=False,
               workload="C5 synthetic |E|=1M DistMult d=256, 8,192 sweeps (wide split-bf16 MFMA filter, "
                        "exact f32 ranks)"),
    "zsl": dict(dataset="FB15K-237-ZS", model="extractor", dim=200, norm=False,
                workload="ZSL eval FB15K-237-ZS: Extractor (d=200, max_neighbor=50) + mean-cosine rank of "
                         "17,596 queries x ~1,000 candidates (SURVEY 8(f) rank 1)"),
    "ns": dict(dataset="FB15K-237-ZS", model="ns", dim=200, norm=True,
               workload="C2 training step FB15K-237-ZS TransE d=200 p=1 norm_flag: OpenKE sampler (B=2,721 positives, "
                        "neg_ent 25, bern) + fused margin loss (MarginLoss 5.0) forward + backward + SGD step"),
    "gan": dict(dataset="FB15K-237-ZS", model="gan", dim=200, norm=False,
                workload="ZSL GAN iteration FB15K-237-ZS (ZSLmodule.train, SURVEY 8(f) rank 3): 1 D step + 1 G step, "
                         "G_batch_size 256 x gan_batch_rela 2 = 512 rows, d=200, 206 seen-relation centroids"),
    "m3ae": dict(dataset="FB15K-237-ZS", model="m3ae", dim=200, norm=False,
                 workload="UnifiedModel.generate over the 235 FB15K-237-ZS relation descriptions x test_sample 20 "
                          "(4,700 rows of 320 tokens): frozen M3AE-small text encoder (d 384, 12 blocks) + SN "
                          "generator + LayerNormalization (SURVEY 8(f) rank 4)"),
}
MFMA_F32_PEAK = 157.3e12  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
MFMA_BF16_PEAK = 16 * MFMA_F32_PEAK  # dense bf16 MFMA: 16x the f32 rate (MI355X_MICROARCH.md, ~2.5 PF)
MFMA_FILTER = os.environ.get("MMRE_MFMA_FILTER", "1") != "0"


def bytes_per_triple(model, dim):
    """algorithmic fp32 bytes of the entity row(s) read per scored triple."""
    return {"transe": 4 * dim, "transe_l2": 4 * dim, "distmult": 4 * dim, "complex": 8 * dim,
            "rotate": 8 * dim}[model]


def valu_ops_per_triple(model, dim, l1_bits=16):
    """VALU issue slots per scored triple in the sweep's inner loop, counted from
    the instruction stream and checked against SQ_INSTS_VALU (profiles/pmc_*.json): TransE L1
    sub + add per element; RotatE 9 per complex element: 5 full-rate f32 ops (dr, di, dr*dr,
    fma(di, di, .), the accumulate) + the raw v_sqrt_f32 of the fast filter at quarter rate =
    4 slots (scripts/probes/trans_rate.hip, rot_rate.hip). The rare exact rescoring of
    undecided pairs is not counted (it is work the filter adds, not the triple's)."""
    if model == "transe" and os.environ.get("MMRE_L1_FILTER", "1") != "0" and l1_bits:
        # the integer filter (mmre_link_sweep_l1q): one v_sad_u16 per two elements at half rate
        # (scripts/probes/sad_rate.hip: 4.64 vs 2.36 cycles per wave-instruction) = 1 slot each;
        # with the 8-bit codes one v_sad_u8 (the same issue cost, scripts/probes/sad8_rate.hip)
        # per four elements = half a slot each
        return dim // 2 if l1_bits == 8 else dim
    return {"transe": 2 * dim, "transe_l2": 3 * dim, "rotate": 9 * dim}.get(model)


# (the VALU sweeps' names without their last template argument: DYNC, the dynamic scheduling's
#  units per claim -- 4, 1, or 0 for the static ranges -- depends on the sweep's size)
KERNEL_NAMES = {"transe": "k_sweep_valu<6, false, false, 0," if os.environ.get("MMRE_L1_FILTER", "1") != "0"
                else "k_sweep_valu<0, false, false, 0,", "rotate": "k_sweep_valu<2, false, false, 3,",
                "distmult": "k_sweep_bf3<2>" if MFMA_FILTER else "k_sweep_mfma<false, false, 2",
                "complex": "k_sweep_bf3<2>" if MFMA_FILTER else "k_sweep_mfma<false, false, 2"}


def pmc_traffic(config: str, model: str):
    """HBM-side bytes per sweep launch from the committed rocprofv3 PMC passes
    (profiles/pmc_<config>.json, made by scripts/pmc.sh + scripts/pmc_summary.py on this
    workload at N=1): (2 x FETCH_SIZE + WRITE_SIZE) KiB -- FETCH_SIZE reads half the bytes of
    wide coalesced loads on gfx950 (MI355X_MICROARCH.md §HBM). Only counters captured on the
    library this process loaded count: the file's __build__.lib_sha256 must equal
    lib_identity()'s, else (None, reason) -- a stale summary is never quoted as traffic.
    Returns (bytes or None, source or reason)."""
    from mmre._lib import lib_identity
    path = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    rel = os.path.relpath(path, REPO)
    sha = (d.get("__build__") or {}).get("lib_sha256")
    mine = lib_identity()["sha256"]
    if sha != mine:
        return None, f"{rel} was captured on libmmre_hip.so {sha or '(unrecorded)'}, not this build ({mine})"
    for name, c in d.items():
        if KERNEL_NAMES[model] in name and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            return (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0, rel
    return None, f"{rel} holds no FETCH_SIZE / WRITE_SIZE of {KERNEL_NAMES[model]}"


def pmc_step_traffic(config: str, kernels):
    """HBM-side bytes of one training step: (2 x FETCH_SIZE + WRITE_SIZE) KiB summed over the
    step's kernels (a substring each) from profiles/pmc_<config>.json, under the same build tie
    as pmc_traffic. Returns (bytes or None, source or reason, per-kernel bytes)."""
    from mmre._lib import lib_identity
    path = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None, None, None
    with open(path) as f:
        d = json.load(f)
    rel = os.path.relpath(path, REPO)
    sha = (d.get("__build__") or {}).get("lib_sha256")
    mine = lib_identity()["sha256"]
    if sha != mine:
        return None, f"{rel} was captured on libmmre_hip.so {sha or '(unrecorded)'}, not this build ({mine})", None
    per = {}
    for k in kernels:
        hits = [c for name, c in d.items() if k in name and "FETCH_SIZE" in c and "WRITE_SIZE" in c]
        if not hits:
            return None, f"{rel} holds no FETCH_SIZE / WRITE_SIZE of {k}", None
        per[k] = (2.0 * hits[0]["FETCH_SIZE"] + hits[0]["WRITE_SIZE"]) * 1024.0
    return sum(per.values()), rel, per


REF_SAMPLE = {"c1": 1000, "c2": 1000, "c3": 1000, "c4": 250, "c5": 250}   # test triples in the CPU leg
REF_NEAR_REL = 1e-5   # the parity block's near-tie window, x max|score| of the sweep (as the fixtures')


def ref_tester_leg(w, n_sample: int, timeout_s: int = 600, reps: int | None = None):
    """The reference's CPU path on this host's cores, as child processes (oracle/ref_tester.py:
    the OpenKE Tester loop with the reference's own Base.so ranker -- oracle/_ref, compiled
    from /root/reference/OpenKE/openke/base/Base.cpp -- and the reference models' predict op
    sequences on torch CPU). The first n_sample test triples (Test.h order) are its test set,
    cut into one contiguous chunk per host thread (ref_tester.run_parallel: one Base.so per
    process, each filtering with the whole filter set). Returns the merged result (per-query
    raw / filtered counts read from Base.so's rank accumulators, the truth's reference score,
    max|score| and the near-tie lists per sweep, the sample's metrics, the slowest chunk's
    time), or None if the reference library is absent or a child fails."""
    ref_so = os.path.join(REPO, "oracle", "_ref", "Base.so")
    if not os.path.exists(ref_so):
        print("cpu_baseline: oracle/_ref/Base.so absent (build() compiles it where /root/reference exists)",
              file=sys.stderr)
        return None
    n = min(int(n_sample), len(w["test_h"]))
    procs = max(1, torch.get_num_threads())
    q = tuple(np.asarray(w[k][:n], np.int64) for k in ("test_h", "test_r", "test_t"))
    try:
        import ref_tester
        out = ref_tester.run_parallel(w, *q, procs, timeout_s=timeout_s, summary=True, near_rel=REF_NEAR_REL)
        # repetitions of the same statistic (whole sample / slowest chunk), so that the reported
        # spread brackets the value: 5 in all when a repetition's loop takes <= 20 s, else 3
        n_reps = reps if reps else (5 if float(out["elapsed"]) <= 20.0 else 3)
        reps = [float(out["elapsed"])]
        while len(reps) < n_reps:
            again = ref_tester.run_parallel(w, *q, procs, timeout_s=timeout_s, summary=True, near_rel=REF_NEAR_REL)
            if not np.array_equal(again["counts"], out["counts"]):
                raise RuntimeError("ref_tester repetition gave different counts")
            reps.append(float(again["elapsed"]))
        out["elapsed_reps"] = np.asarray(reps)
    except Exception as e:  # noqa: BLE001 -- the baseline is reported, never required
        print(f"cpu_baseline: ref_tester failed: {e!r}", file=sys.stderr)
        return None
    out["n"] = n
    return out


def cpu_baseline_block(ref, w):
    E, n = int(ref["n_ent"]), int(ref["n"])
    reps = np.asarray(ref.get("elapsed_reps", [ref["elapsed"]]), np.float64)
    el = float(np.median(reps))  # the median repetition's slowest chunk
    P = int(ref["threads"])
    note = ""
    if w["model"] == "rotate":
        note = (" RotatE: ~99% of the reference's CPU time is torch.norm over the size-2 stacked dim "
                "(RotatE.py:74-75), a CPU pathology of the reference path that inflates GPU/CPU ratios.")
    out = {"value": 2 * n * E / el, "unit": "scored triples/s", "cores": P, "kind": "reference",
           "sample": f"first {n} {w['dataset']} test triples (Test.h order) x {{head,tail}} = {2 * n} sweeps x {E} "
                     f"entities through the OpenKE Tester loop: reference Base.so getHeadBatch/testHead/testTail "
                     f"(oracle/_ref) + the reference {w['model']} predict op sequence on torch {torch.__version__} "
                     f"CPU (oracle/ref_tester.py), {P} processes x 1 thread side by side (contiguous chunks of "
                     f"the sample), slowest chunk {el:.2f} s (median of {len(reps)} repetitions).{note}"}
    # the spread: the same statistic (whole sample / slowest chunk) per repetition
    rates = 2 * n * E / reps
    out.update({"reps": int(len(rates)), "value_min": float(rates.min()), "value_median": float(np.median(rates)),
                "value_max": float(rates.max()),
                "reps_note": f"value = whole sample / slowest chunk of the median repetition; min / median / max of "
                             f"that statistic over {len(rates)} repetitions of the whole leg ({P} processes each; "
                             f"the host share is not isolated: the spread is the box's noise)"})
    return out


def sample_scores(spec, w, n, dev):
    """GPU model.predict values of the sample's 2n sweeps ([head block | tail block], (2n, E)
    on the device): the same query-prep + sweep kernels as the evaluation, with the score
    write-back on."""
    from mmre.link import HEAD, TAIL, LinkSweep
    th, tr, tt = (np.asarray(w[k][:n], np.int64) for k in ("test_h", "test_r", "test_t"))
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    qm = np.concatenate([np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)])
    res = LinkSweep(spec).run(to(np.r_[th, th]), to(np.r_[tr, tr]), to(np.r_[tt, tt]), to(qm), return_scores=True)
    return res["scores"]


def parity_block(ref, counts, n_total, w, gpu_scores, tc: bool = False):
    """GPU per-query counts vs the reference Base.so's on the cpu_baseline sample, query by
    query, as tests/test_ref_fixture_gpu.py checks the fixtures: the reference lists, per
    sweep, every entity whose reference score lies within REF_NEAR_REL x max|score| of the
    truth's; the GPU's own scores of those entities and of the truth (gpu_scores, the
    score-storing sweep) decide their side of Test.h's strict `<` (Test.h:83, :147), and the
    expected GPU count is the reference's moved by exactly the entities whose side differs
    (filtered: unless the entity is a known triple). window_ok: the measured GPU-vs-reference
    error on those scores stays below 1/4 of the window, so no unlisted entity can flip.
    Metrics: the sample's hit@{1,3,10} / MR / MRR from the GPU's counts (the P14 reduction)
    and the reference's (Base.so's Test.h reduction, restated over the merged chunks).
    tc: the type-constrained counts (Test.h's *_constrain counters, type_constrain.txt from
    w["type_heads"] / w["type_tails"]) instead -- a near entity moves them only when its type fits."""
    from mmre.link import link_metrics
    n = int(ref["n"])
    q = ref["q"].astype(np.int64)
    h, r, t = q[:, 0], q[:, 1], q[:, 2]
    same_q = bool(np.array_equal(h, w["test_h"][:n]) and np.array_equal(r, w["test_r"][:n])
                  and np.array_equal(t, w["test_t"][:n]))
    E, R = int(w["n_ent"]), int(w["n_rel"])
    gh = counts[:, :n].T.astype(np.int64)                  # (n, 4) raw, filt, raw_tc, filt_tc
    gt = counts[:, n_total:n_total + n].T.astype(np.int64)
    cols = slice(2, 4) if tc else slice(0, 2)
    gpu_c = np.stack([gh[:, cols], gt[:, cols]])            # (2, n, 2) [head|tail][q][raw, filt] (type-constrained: tc)
    ref_c = ref["counts"].astype(np.int64)[:, :, cols]
    off, ids = ref["near_off"], ref["near_ids"].astype(np.int64)
    sweep_of = np.repeat(np.arange(2 * n), np.diff(off))
    dev = gpu_scores.device
    tt_ = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    truth_ids = np.r_[h, t]
    g_truth = gpu_scores[tt_(np.arange(2 * n)), tt_(truth_ids)].cpu().numpy().astype(np.float64)
    g_near = (gpu_scores[tt_(sweep_of), tt_(ids)].cpu().numpy().astype(np.float64) if len(ids)
              else np.zeros(0, np.float64))
    r_truth = ref["truth_scores"].reshape(-1).astype(np.float64)
    r_near = ref["near_scores"].astype(np.float64)
    err = np.abs(g_truth - r_truth)
    if len(ids):
        np.maximum.at(err, sweep_of, np.abs(g_near - r_near))
    window = REF_NEAR_REL * ref["score_absmax"].reshape(-1).astype(np.float64)
    flip = (g_near < g_truth[sweep_of]).astype(np.int64) - (r_near < r_truth[sweep_of]).astype(np.int64)
    head = sweep_of < n
    qi = np.where(head, sweep_of, sweep_of - n)
    key = lambda a, b, c: (a * R + b) * E + c
    known_keys = np.unique(key(np.asarray(w["filter_h"], np.int64), np.asarray(w["filter_r"], np.int64),
                               np.asarray(w["filter_t"], np.int64)))
    known = np.isin(np.where(head, key(ids, r[qi], t[qi]), key(h[qi], r[qi], ids)), known_keys)
    if tc:  # only a near entity of the relation's type moves the constrained counts
        tkey = lambda rr, e: rr * E + e
        types = [np.unique(np.concatenate([tkey(np.int64(rr), np.asarray(lst, np.int64)) for rr, lst in
                                           enumerate(w[name])] + [np.zeros(0, np.int64)]))
                 for name in ("type_heads", "type_tails")]
        ok = np.where(head, np.isin(tkey(r[qi], ids), types[0]), np.isin(tkey(r[qi], ids), types[1]))
        flip = flip * ok
    d_raw = np.bincount(sweep_of, weights=flip, minlength=2 * n).astype(np.int64).reshape(2, n)
    d_filt = np.bincount(sweep_of, weights=flip * (~known), minlength=2 * n).astype(np.int64).reshape(2, n)
    expect = ref_c + np.stack([d_raw, d_filt], axis=2)
    mism = gpu_c != ref_c
    gm = link_metrics(counts[:, :n], counts[:, n_total:n_total + n])["filter_tc" if tc else "filter"]
    rm = ref["metrics"]  # MRR, MR, hit10, hit3, hit1 (filter, or filter_tc with tc; Test.h:232-327)
    gpu_vals = np.array([gm["mrr"], gm["mr"], gm["hit10"], gm["hit3"], gm["hit1"]], np.float32)
    return {"source": f"reference Base.so Tester loop on the cpu_baseline sample (oracle/ref_tester.py, "
                      f"{int(ref['threads'])} chunks)" + (", type-constrained counts (testHead/testTail with "
                                                          "type_constrain, importTypeFiles)" if tc else ""),
            "test_triples": n, "sweeps": 2 * n, "queries_match": same_q,
            "tie_window": f"{REF_NEAR_REL} x max|s_ref| per sweep (the reference's near lists)",
            "score_err_max": float(err.max()), "window_ok": bool(np.all(err <= 0.25 * window)),
            "raw_mismatches": int(mism[:, :, 0].sum()), "filt_mismatches": int(mism[:, :, 1].sum()),
            "unexplained_mismatches": int((gpu_c != expect).sum()), "near_tie_sweeps": int((np.diff(off) > 0).sum()),
            "hit1_gpu": float(gm["hit1"]), "hit3_gpu": float(gm["hit3"]), "hit10_gpu": float(gm["hit10"]),
            "mr_gpu": float(gm["mr"]), "mrr_gpu": float(gm["mrr"]),
            "hit1_ref": float(rm[4]), "hit3_ref": float(rm[3]), "hit10_ref": float(rm[2]), "mr_ref": float(rm[1]),
            "mrr_ref": float(rm[0]),
            "metrics_bit_equal": bool(np.array_equal(gpu_vals.view(np.uint32), rm.astype(np.float32).view(np.uint32)))}


def cpu_baseline_zsl(w, budget_s: float = 15.0, max_queries: int = 400):
    """ZSLmodule.eval's per-query loop on the host cores (zsl_module.py:666-706): get_meta,
    Extractor forward on torch CPU (the oracle's op-for-op restatement, eval mode), sklearn
    cosine_similarity(...).mean(1), argsort rank; queries in order until the time budget."""
    import zsl_extractor as ox
    from sklearn.metrics.pairwise import cosine_similarity
    d = w["dim"]
    ref = ox.ExtractorRef(d, w["n_sym"], w["sym_emb"].numpy())
    gen = torch.Generator().manual_seed(0)
    with torch.no_grad():
        for name, p in ref.named_parameters():
            if p.dim() == 2 and not name.startswith("symbol_emb"):
                p.copy_(torch.nn.init.xavier_normal_(torch.empty(p.shape), generator=gen))
            elif name.endswith("bias"):
                p.zero_()
    off, ch, ct = w["off"], w["cand_head"], w["cand_tail"]
    rv = w["rel_vecs"].numpy()
    conn, deg, es = w["conn"], w["deg"], w["ent_sym"]
    rows = 0
    t0 = time.perf_counter()
    q = 0
    while q < min(max_queries, len(off) - 1) and time.perf_counter() - t0 < budget_s:
        a, b = off[q], off[q + 1]
        left, right = ch[a:b], ct[a:b]
        pairs = torch.from_numpy(np.stack([es[left], es[right]], 1))
        meta = (torch.LongTensor(np.stack([conn[i] for i in left])), torch.FloatTensor(deg[left]),
                torch.LongTensor(np.stack([conn[i] for i in right])), torch.FloatTensor(deg[right]))
        vecs, _ = ref(pairs, pairs, meta, meta)
        scores = cosine_similarity(vecs.numpy(), rv[w["query_set"][q]]).mean(axis=1)
        list(np.argsort(scores))[::-1].index(0)
        rows += b - a
        q += 1
    el = time.perf_counter() - t0
    return {"value": rows / el, "unit": "scored candidates/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"first {q} FB15K-237-ZS ZSL queries ({rows} candidate rows) through the ZSLmodule.eval loop "
                      f"(oracle/zsl_extractor.py: torch {torch.__version__} CPU Extractor + sklearn cosine + argsort),"
                      f" {el:.2f} s on {torch.get_num_threads()} threads"}


def bench_zsl(args, world, rank, dev, dist):
    """One step = one full ZSL evaluation (ZSLmodule.eval, zsl_module.py:635-745) of this rank's
    relation shard: weight pack + per-entity node tables, normalised mean relation vectors, the
    fused Extractor/SupportEncoder/cosine kernel over every candidate row, the descending rank,
    (N>1) the all-gather of ranks, D2H and Hits@10/5/1 + MRR on the host."""
    from mmre.extractor import encode, node_tables, pack_weights, rank_desc, targets
    from mmre.sharding import lpt_partition
    from mmre.workloads import zsl_workload
    from module.zsl_module import Extractor, weights_init
    w = zsl_workload(dim=CONFIGS["zsl"]["dim"])
    d = w["dim"]
    torch.manual_seed(0)
    ex = Extractor(d, w["n_sym"], w["sym_emb"].numpy())
    ex.apply(weights_init)
    ex = ex.to(dev).eval()
    nq = len(w["off"]) - 1
    masks = lpt_partition(w["query_rel"], world)
    mine = np.nonzero(masks[rank])[0]
    off = w["off"]
    lens = off[mine + 1] - off[mine]
    rows = np.concatenate([np.arange(off[q], off[q + 1]) for q in mine]) if len(mine) else np.zeros(0, np.int64)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ch, ct = to(w["cand_head"][rows]), to(w["cand_tail"][rows])
    loff = to(np.r_[0, np.cumsum(lens)].astype(np.int64))
    row_set = to(np.repeat(w["query_set"][mine], lens))
    ent_sym, conn, deg = to(w["ent_sym"]), to(w["conn"]), to(w["deg"])
    rel_vecs = w["rel_vecs"].to(dev)
    n_rows = int(len(rows))
    pad = max(int(m.sum()) for m in masks)
    host = torch.empty(world * pad, dtype=torch.int32, pin_memory=True)

    def step(ev=None):
        pack = pack_weights(ex)
        left, right = node_tables(pack, d, ex.symbol_emb.weight, ent_sym, conn, deg)
        t = targets(rel_vecs, normalize=True)
        if ev:
            ev[0].record()
        _, s = encode(pack, d, ex.support_encoder.layer_norm.eps, left, ch, right, ct, targets=t,
                      row_target=row_set, normalize=True)
        if ev:
            ev[1].record()
        r = rank_desc(s, loff)
        if dist:
            buf = torch.zeros(pad, dtype=torch.int32, device=dev)
            buf[:len(mine)] = r
            out = torch.empty(world * pad, dtype=torch.int32, device=dev)
            dist.all_gather_into_tensor(out, buf)
            r = out
        host[:r.numel()].copy_(r, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        got = host.numpy()
        full = np.empty(nq, np.int64)
        for k in range(world):
            ids = np.nonzero(masks[k])[0]
            full[ids] = got[k * pad:k * pad + len(ids)]
        return {"hits10": float((full <= 10).mean()), "hits5": float((full <= 5).mean()),
                "hits1": float((full <= 1).mean()), "mrr": float((1.0 / full).mean())}

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = None
    for i in range(args.steps):
        m = step(evs[i])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=_coll_dev(dist, dev))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total = int(off[-1])
    if rank == 0:
        flops = 8.0 * d * d * n_rows  # proj1 (d -> 2d) + proj2 (2d -> d), 2 flops per MAC
        ach = flops / (kern_ms * 1e-3) / 1e12
        out = {"metric": f"scored candidates/sec, {CONFIGS['zsl']['workload']}", "value": total * args.steps / elapsed,
               "unit": "scored candidates/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
               "vs_baseline": None, "dtype": "f32",
               "data": "real FB15K-237-ZS test triples + rel2candidates_all pools; synthetic train neighbourhoods, "
                       "random-init Extractor (weights_init) and relation vectors",
               "config": {"workload": CONFIGS["zsl"]["workload"], "n_queries": nq, "n_candidate_rows": total,
                          "dim": d, "max_neighbor": w["max_nb"],
                          "parallelism": f"relation-sharded x{world} (LPT), RCCL all-gather of ranks"},
               "roofline": {"bound": "mfma", "achieved": ach, "peak": MFMA_F32_PEAK / 1e12, "unit": "TFLOP/s",
                            "frac": ach * 1e12 / MFMA_F32_PEAK, "traffic": None,
                            "kernel": "k_extractor_encode<200>", "kernel_ms": kern_ms,
                            "flops_per_row": 8 * d * d, "rows_per_launch": n_rows},
               "metrics": m}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_zsl(w)
        print(json.dumps(_with_build(out)), flush=True)
    if dist:
        dist.destroy_process_group()


def bench_ns(args, world, rank, dev, dist):
    """One step = one OpenKE training step at the C2 training shape (Trainer.train_one_step,
    Trainer.py:43-54, over the loader's Base.cpp sampling): a bit-exact GPU sampler batch
    (mmre.sampler.OpenKESampler: B = 2,721 positives x (1 + neg_ent) rows, bern), the fused
    negative-sampling margin loss forward + backward into the dense tables (mmre.ns), SGD.
    Training triples = the C2 filter set (272,115 synthetic + the test triples). N > 1: data
    parallel replicas (each rank its own sampler stream; no gradient exchange is timed)."""
    import ref_trainer  # noqa: F401  (import check of the CPU leg before timing)
    from mmre.data import TrainIndex
    from mmre.ns import NSSpec, fused_ns_loss
    from mmre.sampler import OpenKESampler
    from mmre.workloads import zs_workload
    model = args.ns_model
    w = zs_workload("FB15K-237-ZS", model, 200)
    E, R, d = w["n_ent"], w["n_rel"], w["dim"]
    B, k, margin = 2721, args.ns_neg, 5.0
    idx = TrainIndex(w["filter_h"], w["filter_t"], w["filter_r"], E, R)
    smp = OpenKESampler(idx, dev, bern=True, seed_skip=8 * rank)
    ent = w["ent"].to(dev).requires_grad_(True)
    rel = w["rel"].to(dev).requires_grad_(True)
    ent_im = w["ent_im"].to(dev).requires_grad_(True) if "ent_im" in w else None
    rel_im = w["rel_im"].to(dev).requires_grad_(True) if "rel_im" in w else None
    if model == "transe":
        spec = NSSpec("transe", d, norm_flag=True)
    elif model == "rotate":  # OpenKE RotatE (margin 6, epsilon 2): the model's own margin transform
        from mmre.link import rotate_phase_denom
        spec = NSSpec("rotate", d, model_margin=6.0, phase_denom=rotate_phase_denom(6.0, 2.0, d))
    else:
        spec = NSSpec(model, d)
    tables = [x for x in (ent, rel, ent_im, rel_im) if x is not None]
    from mmre.optim import SGD
    opt = SGD(tables, lr=1.0)  # OpenKE Trainer's optimizer: one HIP launch per step
    n_rows = B * (1 + k)
    bufs = [dict(batch_h=torch.empty(n_rows, dtype=torch.int64, device=dev),
                 batch_t=torch.empty(n_rows, dtype=torch.int64, device=dev),
                 batch_r=torch.empty(n_rows, dtype=torch.int64, device=dev),
                 batch_y=torch.empty(n_rows, dtype=torch.float32, device=dev)) for _ in range(2)]

    tstep = None
    if not args.ns_autograd:
        # the whole step as ONE C-ABI call, pipelined (TransE: mmre_ns_step_openke_pipe -- the fused
        # loss kernel, the row owner with SGD, the loss reduction, the next batch and the updated
        # rows' pre-pass; DistMult / ComplEx / RotatE: mmre_ns_step_openke_gen_pipe -- forward, slot
        # records, row owner with SGD, the loss reduction and the next batch), bit-identical to the
        # drop-in path below (tests/test_ns_full_gpu.py::test_*train_step_equals_the_autograd_path)
        from mmre.ns import OpenKETrainStep
        tstep = OpenKETrainStep(smp, spec, ent, rel, B, k, margin, 1.0, ent_im=ent_im, rel_im=rel_im)

    def step(i, ev=None):
        if tstep is not None:
            if ev:
                for e in ev[:4]:
                    e.record()
            loss = tstep()
            if ev:
                for e in ev[4:]:
                    e.record()
            return loss
        b = smp.sample(B, k, out=bufs[i & 1])
        opt.zero_grad(set_to_none=True)
        if ev:
            ev[0].record()
        loss, _ = fused_ns_loss(spec, ent, rel, b["batch_h"], b["batch_t"], b["batch_r"], B, k, margin,
                                events=ev[3:7] if ev else None, optimizer=opt, ent_im=ent_im, rel_im=rel_im)
        if ev:
            ev[1].record()
        loss.backward()
        if ev:
            ev[2].record()
        opt.step()
        return loss

    # warmup on a side stream (lazy autograd / optimizer state), then -- unless --ns-eager -- the
    # whole training step (sampler batch + device seed advance, fused loss and gradients, the
    # autograd backward, SGD) captured once into a hipGraph and replayed: the step's ~12 launches
    # cost one, and nothing waits for the host (the sampler keeps its LCG states in HBM)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for i in range(args.warmup):
            step(i)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    graph = None
    one = torch.ones((), dtype=torch.float32, device=dev)  # the upstream gradient loss.backward() would fill
    if not args.ns_eager:
        # two hipGraphs, one per batch buffer: graph p trains on bufs[p] while a forked stream
        # samples the next batch into bufs[1 - p] (the data loader's prefetch: the sampler's
        # batches and LCG states are the serial sequence, batch i + 1 drawn after batch i), then
        # joins. --ns-serial: one graph, the batch sampled in line before the step.
        graphs = []
        fork = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream(dev)
        for par in ((0,) if (not args.ns_prefetch and tstep is None) else (0, 1)):
            opt.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if tstep is not None:  # the one-call step (no prefetch variant)
                    g_loss, g_b = tstep(), None
                else:
                    if (not args.ns_prefetch):
                        g_b = smp.sample(B, k, out=bufs[0])
                    else:
                        g_b = bufs[par]
                        fork.wait_stream(torch.cuda.current_stream(dev))
                        with torch.cuda.stream(fork):
                            smp.sample(B, k, out=bufs[1 - par])
                    g_loss, _ = fused_ns_loss(spec, ent, rel, g_b["batch_h"], g_b["batch_t"], g_b["batch_r"], B, k,
                                              margin, optimizer=opt, ent_im=ent_im, rel_im=rel_im)
                    torch.autograd.backward(g_loss, grad_tensors=one)
                    opt.step()
                    if not (not args.ns_prefetch):
                        torch.cuda.current_stream(dev).wait_stream(fork)
            graphs.append(g)
            if tstep is not None and (not tstep.pipeline or len(graphs) == 2):
                break  # the pipelined one-call step: one graph per parity, replayed alternately
        graph = graphs[0]
        if not (not args.ns_prefetch):
            smp.sample(B, k, out=bufs[0])  # the first batch; every replay then prefetches the next
        torch.cuda.synchronize()
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(7)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if graph is not None:
            graphs[i % len(graphs)].replay()
        else:
            loss = step(i, evs[i])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    pipe_ms = None
    if graph is not None and tstep is not None and tstep.pipeline:
        # the pipelined step's two launches (fused loss kernel; row owner with SGD, the loss, the
        # next batch's sampler and the updated rows' pre-pass): events around replays of its graphs
        pev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for i, (a_, b_) in enumerate(pev):
            a_.record()
            graphs[(args.steps + i) % 2].replay()
            b_.record()
        torch.cuda.synchronize()
        pipe_ms = float(np.mean([a_.elapsed_time(b_) for a_, b_ in pev]))
    if tstep is not None and graph is not None:
        tstep.invalidate()  # the replays advanced the device state past the step object's record
    if graph is not None:  # the fused call and the step's parts timed on eager steps after the timed region
        loss = g_loss.detach().clone()
        del g_loss, g_b, graph, graphs  # drop the captured autograd graphs before eager backward passes
        graph = True
        evs = evs[:20]
        for i in range(len(evs)):
            step(i, evs[i])
        torch.cuda.synchronize()
    fwd_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    bwd_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    fused_fwd_ms = float(np.mean([e[3].elapsed_time(e[4]) for e in evs]))
    fused_grad_ms = float(np.mean([e[5].elapsed_time(e[6]) for e in evs]))
    # the fused loss + gradient alone, as the step runs it (graph-replayed, no launch gaps): the
    # one-shot C-ABI call mmre_ns_forward_backward captured in a hipGraph, events around replays
    from mmre._lib import call, lib, ptr, stream_ptr
    g_in = smp.sample(B, k, out=bufs[0])
    wk = torch.empty(int(lib().mmre_ns_fused_workspace(spec.model_id, int(spec.norm_flag), B, k, E, R, d)),
                     dtype=torch.float32, device=dev)
    s1 = torch.empty(n_rows, dtype=torch.float32, device=dev)
    l1 = torch.empty(1, dtype=torch.float32, device=dev)
    ge, gr = torch.empty_like(ent), torch.empty_like(rel)
    gei = torch.empty_like(ent_im) if ent_im is not None else None
    gri = torch.empty_like(rel_im) if rel_im is not None else None
    e0, r0 = ent.detach(), rel.detach()
    ei0 = ent_im.detach() if ent_im is not None else None
    ri0 = rel_im.detach() if rel_im is not None else None

    def one_shot():
        call("mmre_ns_forward_backward", spec.model_id, int(spec.norm_flag), spec.model_margin,
             int(spec.use_model_margin), ptr(e0), ptr(ei0), ptr(r0), ptr(ri0), E, R, d, spec.phase_denom,
             ptr(g_in["batch_h"]), ptr(g_in["batch_t"]), ptr(g_in["batch_r"]), B, k, margin, 0.0, 0.0,
             ptr(s1), ptr(l1), ptr(ge), ptr(gei), ptr(gr), ptr(gri), ptr(wk), stream_ptr(dev))
    one_shot()
    torch.cuda.synchronize()
    g_fused = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_fused):
        one_shot()
    fev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a_, b_ in fev:
        a_.record()
        g_fused.replay()
        b_.record()
    torch.cuda.synchronize()
    fused_ms = float(np.mean([a_.elapsed_time(b_) for a_, b_ in fev]))
    del g_fused, wk
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=_coll_dev(dist, dev))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank == 0:
        # a gather-bound HBM path. Algorithmic bytes: forward = B*3*4d (positive h, r,
        # t) + B*k*4d (one corrupted row per negative) + B(1+k)*3*8 (int64 ids); gradient = the
        # dense gradient tables written once, (E + R)*4d. The implementation also moves its slots,
        # written by the fused kernel and read back by the row-owner pass: three d-float sum rows
        # per positive, a 72-B sign record per negative (L1, d 200: |g| + two 4 x 64-bit planes),
        # and per slot a key, an occurrence count and a bucketed id: slot_bytes.
        if model == "transe":
            fwd_bytes = B * 3 * 4 * d + B * k * 4 * d + n_rows * 3 * 8
            grad_bytes = (E + R) * 4 * d
            slot_bytes = 2 * (B * 3 * 4 * d + B * k * 4 * (2 + 4 * 4)) + 2 * 3 * 4 * B * (3 + 3 * k)
        else:  # k_ns_forward reads the three rows of every batch row; records of 2 d_pad floats per slot
            eb = 4 * d * (2 if model in ("complex", "rotate") else 1)
            rb = 4 * d * (2 if model == "complex" else 1)
            fwd_bytes = n_rows * (2 * eb + rb) + n_rows * 3 * 8
            grad_bytes = E * eb + R * rb
            slot_bytes = 2 * (B * (3 + 3 * k)) * 2 * 4 * (256 if d > 128 else 128)
        kern_ms = pipe_ms if pipe_ms is not None else fused_ms
        ach = (fwd_bytes + grad_bytes) / (kern_ms * 1e-3) / 1e9
        if model == "transe":
            step_kernels = (["k_ns_transe_fused<4, false, false>", "k_ns_row_owner<4, false>"] if pipe_ms is not None
                            else ["k_ns_prepass(", "k_ns_transe_fused<4, false, false>", "k_ns_reduce(",
                                  "k_ns_row_owner<4, false>"])
        else:
            step_kernels = (["k_ns_gen_forward<4, ", "k_ns_gen_slots<4, ", "k_ns_gen_owner<4>"] if pipe_ms is not None
                            else ["k_ns_gen_forward<4, ", "k_ns_reduce(", "k_ns_gen_slots<4, ", "k_ns_gen_owner<4>"])
        pmc_cfg = "ns" if model == "transe" else f"ns_{model}"  # profiles/pmc_<pmc_cfg>.json
        traffic, tsrc, tper = (pmc_step_traffic(pmc_cfg, step_kernels) if (world == 1 and d == 200 and k == 25)
                               else (None, None, None))
        out = {"metric": f"training triples/sec, {CONFIGS['ns']['workload']}",
               "value": n_rows * args.steps * world / elapsed, "unit": "training triples/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": f"synthetic {model} tables (OpenKE init, seed 0); training triples = 272,115 synthetic "
                       "+ the FB15K-237-ZS test triples",
               "config": {"workload": CONFIGS["ns"]["workload"] if model == "transe" else
                          f"{model} d=200 training step at the C2 training shape (margin loss)", "model": model,
                          "batch": B, "neg_ent": k, "rows_per_step": n_rows,
                          "dim": d, "margin": margin, "parallelism": f"data-parallel replicas x{world}",
                          "step": (("mmre_ns_step_openke_pipe (fused loss kernel; row owner + SGD + loss reduction "
                                    "+ the next batch's sampler + the updated rows' pre-pass: 2 launches)" if model == "transe"
                                    else "mmre_ns_step_openke_gen_pipe (forward; slot records; row owner + SGD + loss "
                                    "reduction + the next batch's sampler: 3 launches)")
                                   if tstep is not None and tstep.pipeline else
                                   "mmre_ns_step_openke (sampler + pre-pass, fused loss, row owner + SGD + loss "
                                   "reduction: 3 launches)" if tstep is not None else
                                   "sampler.sample + fused_ns_loss + backward + SGD.step (drop-in path)"),
                          "launch": ("eager" if not graph else "hipGraph replay of the whole step" +
                                     ("" if (not args.ns_prefetch) else ", next batch sampled on a forked stream (prefetch)"))},
               "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                            "traffic_unit": "HBM bytes per step's loss + gradient kernels (rocprofv3 PMC, "
                                            "2 x FETCH_SIZE + WRITE_SIZE)",
                            "traffic_source": tsrc, "traffic_per_kernel": tper,
                            "traffic_x_algorithmic": (traffic / (fwd_bytes + grad_bytes)) if traffic else None,
                            "kernel": (("mmre_ns_step_openke_pipe = k_ns_transe_fused<4, false, false> + "
                                        "k_ns_row_owner<4, false> (+ the loss reduction, the next batch's sampler "
                                        "workgroups and the updated rows' pre-pass in its grid)" if model == "transe" else
                                        "mmre_ns_step_openke_gen_pipe = k_ns_gen_forward + k_ns_gen_slots + "
                                        "k_ns_gen_owner (+ the loss reduction and the next batch's sampler workgroups "
                                        "in its grid)") + ": events around hipGraph replays of the step (one graph per "
                                       "parity)" if pipe_ms is not None else
                                       ("mmre_ns_forward_backward = k_ns_prepass + k_ns_transe_fused<4, false, false> + "
                                        "k_ns_reduce (the loss) + k_ns_row_owner<4, false>" if model == "transe" else
                                        "mmre_ns_forward_backward = k_ns_forward + k_ns_reduce + k_ns_gen_slots + "
                                        "k_ns_gen_owner") + ": events around hipGraph replays of the one-shot C-ABI call"),
                            "kernel_ms": kern_ms, "forward_backward_ms": fused_ms, "eager_fused_forward_ms": fused_fwd_ms,
                            "eager_fused_grad_ms": fused_grad_ms,
                            "algorithmic_bytes": fwd_bytes + grad_bytes, "slot_bytes": slot_bytes,
                            "implementation_frac": (fwd_bytes + grad_bytes + slot_bytes) / (kern_ms * 1e-3)
                                                   / (HBM_PEAK_GBS * 1e9),
                            "step_forward_ms": fwd_ms, "step_backward_ms": bwd_ms,
                            "note": "no float atomics: the gradient contributions are bucketed by table row and "
                                    "one wave per table row summing them in batch order (bit-reproducible); the "
                                    "TransE step is two launches (mmre_ns_step_openke_pipe): the fused loss kernel, the "
                                    "row-owner pass with the SGD step, the loss reduction, the NEXT batch's sampler and "
                                    "the pre-pass of the rows it updates folded in (a prefetching loader; the first step "
                                    "adds the sampler + pre-pass launch) -- bit-identical to mmre_ns_step_openke's three "
                                    "and the drop-in path's five (--ns-autograd)"},
               "last_loss": float(loss.detach())}
        if world == 1 and not args.no_cpu_baseline and model == "transe":
            out["cpu_baseline"] = ref_trainer_leg(w, B, k, margin)
        print(json.dumps(_with_build(out)), flush=True)
    if dist:
        dist.destroy_process_group()


def ref_trainer_leg(w, B, k, margin, steps=30, timeout_s=600, reps=5):
    """The reference's training step on this host's cores (oracle/ref_trainer.py in a child
    process): reference Base.so sampling + the TransE / strategy / MarginLoss op sequence on
    torch CPU + backward + SGD, `steps` steps on the same training triples, the whole leg
    repeated `reps` times: value = the median repetition's rate, value_min / _max the spread of
    that same statistic (so the reported value lies inside its own bracket)."""
    import shutil
    import subprocess
    ref_so = os.path.join(REPO, "oracle", "_ref", "Base.so")
    if not os.path.exists(ref_so):
        return None
    tmp = tempfile.mkdtemp(prefix="mmre_reftrain_")
    runs = []
    try:
        trn = np.stack([w["filter_h"], w["filter_t"], w["filter_r"]], 1)
        with open(os.path.join(tmp, "train2id.txt"), "w") as f:
            f.write(f"{len(trn)}\n")
            np.savetxt(f, trn, fmt="%d")
        for name, cnt in (("entity2id.txt", w["n_ent"]), ("relation2id.txt", w["n_rel"])):
            with open(os.path.join(tmp, name), "w") as f:
                f.write(f"{cnt}\n")
        meta = dict(dim=w["dim"], batch=B, neg=k, margin=margin, norm_flag=True, bern=True, steps=steps,
                    threads=torch.get_num_threads(), sampler_threads=8)
        with open(os.path.join(tmp, "meta.json"), "w") as f:
            json.dump(meta, f)
        for _ in range(reps):
            r = subprocess.run([sys.executable, os.path.join(REPO, "oracle", "ref_trainer.py"), tmp], cwd=REPO,
                               capture_output=True, text=True, timeout=timeout_s)
            if r.returncode != 0:
                print(f"cpu_baseline: ref_trainer failed (rc {r.returncode}): {r.stderr[-800:]}", file=sys.stderr)
                return None
            with open(os.path.join(tmp, "result.json")) as f:
                runs.append(json.load(f))
    except subprocess.TimeoutExpired:
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    rates = [x["rows_per_step"] * x["steps"] / x["elapsed"] for x in runs]
    order = sorted(range(len(runs)), key=lambda i: rates[i])
    res = runs[order[len(order) // 2]]  # the median repetition
    el = res["elapsed"]
    tm = res["times"]
    return {"value": rates[order[len(order) // 2]], "unit": "training triples/s", "cores": res["threads"],
            "kind": "reference",
            "sample": f"{res['steps']} training steps of B={B} x (1+{k}) rows: reference Base.so sampling (8 pthreads) "
                      f"+ TransE/NegativeSampling/MarginLoss op sequence on torch {torch.__version__} CPU + backward + "
                      f"SGD (oracle/ref_trainer.py), {el:.2f} s on {res['threads']} threads (sampling "
                      f"{tm['sampling']:.2f} s, forward {tm['forward']:.2f} s, backward+step {tm['backward_step']:.2f} s; "
                      f"the median of {len(runs)} repetitions)",
            "reps": len(runs), "value_min": min(rates), "value_median": rates[order[len(order) // 2]],
            "value_max": max(rates),
            "reps_note": f"min / median / max of the leg's rate over {len(runs)} repetitions of the whole leg (the "
                         "host share is not isolated: the spread is the box's noise)"}


def bench_gan(args, world, rank, dev, dist):
    """One step = one GAN iteration of ZSLmodule.train (zsl_module.py:417-600) at the reference's
    batch (G_batch_size 256 x gan_batch_rela 2): a Discriminator step (Extractor vectors of the
    real and false pairs, generator in eval mode, 3 + 1 Discriminator calls with spectral-norm
    power iterations, gradient penalty double backward, Adam) and a Generator step (generator
    with power iteration + HIP backward, 3 Discriminator calls, visual-pivot loss, Adam), each
    replayed from its hipGraph with noise / alpha drawn inside the graph."""
    from mmre.extractor import ZSLRanker, encode
    from mmre.gan import ZSLGANStep
    from mmre.generator import RelationGenerator
    from mmre.workloads import zsl_workload
    from module.zsl_module import Discriminator, Extractor, weights_init
    if world > 1:
        raise SystemExit("bench --config gan is a single-GPU step (the GAN trains one model per process)")
    w = zsl_workload(dim=200)
    d, E = w["dim"], w["n_ent"]
    torch.manual_seed(0)
    ex = Extractor(d, w["n_sym"], w["sym_emb"].numpy())
    ex.apply(weights_init)
    ex = ex.to(dev).eval()
    ranker = ZSLRanker(ex, w["ent_sym"], w["conn"], w["deg"], device=dev)
    n_lab = 206
    rng = np.random.default_rng(0)
    # centroids: mean Extractor vector of 256 pairs per seen relation (zsl_module.py:371-383)
    ph = torch.as_tensor(rng.integers(0, E, n_lab * 256), device=dev)
    pt = torch.as_tensor(rng.integers(0, E, n_lab * 256), device=dev)
    g, _ = encode(ranker.pack, d, ranker.ln_eps, ranker.left, ph, ranker.right, pt, want_g=True, want_score=False)
    centroids = g.view(n_lab, 256, d).mean(1)
    gen = RelationGenerator(384, 15, d).to(dev)
    disc = Discriminator(dim=d).to(dev)
    disc.apply(weights_init)
    cls_table = torch.randn(w["n_rel"], 384, device=dev)
    step = ZSLGANStep(gen, disc, cls_table, centroids, ranker, lr_G=1e-4, lr_D=1e-4, pretrain_margin=5.0,
                      gan_batch_rela=2)
    n = 512

    def batch():
        lab = np.repeat(rng.choice(n_lab, 2, replace=False), 256)
        return {k: torch.as_tensor(v, device=dev) for k, v in dict(
            rel=rng.integers(0, w["n_rel"], n), q_head=rng.integers(0, E, n), q_tail=rng.integers(0, E, n),
            f_head=rng.integers(0, E, n), f_tail=rng.integers(0, E, n), labels=lab).items()}

    b0 = batch()
    step.replay("d", b0)  # eager first step + capture
    step.replay("g", b0)

    def one(bt):
        step.replay("d", bt)
        return step.replay("g", bt)

    batches = [batch() for _ in range(args.warmup + args.steps)]
    for i in range(args.warmup):
        one(batches[i])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = one(batches[args.warmup + i])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the same iteration launched eagerly (no graph), for the launch-overhead comparison
    torch.cuda.synchronize()
    te = time.perf_counter()
    k_e = max(3, args.steps // 4)
    for i in range(k_e):
        bt = batches[i]
        noise = torch.randn(n, 15, device=dev)
        alpha = torch.rand(n, 1, device=dev)
        step.d_step(bt["rel"], bt["q_head"], bt["q_tail"], bt["f_head"], bt["f_tail"], bt["labels"], noise, alpha)
        step.g_step(bt["rel"], bt["q_head"], bt["q_tail"], bt["f_head"], bt["f_tail"], bt["labels"], noise)
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - te) / k_e * 1e3
    res = {"metric": f"GAN iterations/sec, {CONFIGS['gan']['workload']}", "value": args.steps / elapsed,
           "unit": "iterations/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32",
           "data": "real FB15K-237-ZS entity graph (synthetic train neighbourhoods), random-init Extractor / "
                   "generator / Discriminator (weights_init), random relation CLS rows and batches",
           "config": {"workload": CONFIGS["gan"]["workload"], "rows": n, "dim": d, "centroids": n_lab,
                      "parallelism": "single GPU, hipGraph replay per D / G step"},
           "eager_ms_per_step": eager_ms, "last_losses_G": [float(x) for x in out.cpu()]}
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_gan(w, centroids.cpu(), n_lab)
    print(json.dumps(_with_build(res)), flush=True)


def cpu_baseline_gan(w, centroids, n_lab, iters=3):
    """The reference's GAN iteration on the host cores: Extractor forwards of the 4 x 512 real /
    false pairs (oracle/zsl_extractor.py, eval) + one D step and one G step (oracle/zsl_gan.py
    GANRef in float32: the op sequence of zsl_module.py:419-600)."""
    import zsl_extractor as ox
    import zsl_gan as og
    from mmre.generator import RelationGenerator
    from module.zsl_module import Discriminator
    d, E = w["dim"], w["n_ent"]
    ref = ox.ExtractorRef(d, w["n_sym"], w["sym_emb"].numpy())
    gen, disc = RelationGenerator(384, 15, d), Discriminator(dim=d)
    D = {k: v.detach().clone() for k, v in disc.state_dict().items()}
    for k in D:
        if not (k.endswith("weight_u") or k.endswith("weight_v")):
            D[k].requires_grad_(True)
    layers = [(L.weight_orig.detach().clone().requires_grad_(), L.bias.detach().clone().requires_grad_(),
               L.weight_u.clone(), L.weight_v.clone())
              for L in (gen.generate_fc_layer, gen.des_rel_map_layer1, gen.des_rel_map_layer2)]
    G = (layers, gen.ln_a.detach().clone().requires_grad_(), gen.ln_b.detach().clone().requires_grad_())
    gan = og.GANRef(D, G, centroids.float())
    rng = np.random.default_rng(1)
    conn, deg, es = w["conn"], w["deg"], w["ent_sym"]
    n = 512

    def vecs(h, t):
        pairs = torch.from_numpy(np.stack([es[h], es[t]], 1))
        meta = (torch.LongTensor(conn[h]), torch.FloatTensor(deg[h]), torch.LongTensor(conn[t]),
                torch.FloatTensor(deg[t]))
        with torch.no_grad():
            return ref.encode(pairs, meta)

    t0 = time.perf_counter()
    for _ in range(iters):
        lab = torch.as_tensor(np.repeat(rng.choice(n_lab, 2, replace=False), 256))
        cls_rows = torch.randn(n, 384)
        for step in ("d", "g"):
            h, t, fh, ft = (rng.integers(0, E, n) for _ in range(4))
            real, neg = vecs(h, t), vecs(fh, ft)
            if step == "d":
                gan.d_step(cls_rows, real, neg, lab, torch.randn(n, 15), torch.rand(n, 1))
            else:
                gan.g_step(cls_rows, real, neg, lab, torch.randn(n, 15))
    el = time.perf_counter() - t0
    return {"value": iters / el, "unit": "iterations/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{iters} GAN iterations (torch {torch.__version__} CPU fp32: oracle Extractor + GANRef "
                      f"D/G steps), {el:.2f} s on {torch.get_num_threads()} threads"}


def _generator_cpu(gen, cls, noise):
    """UnifiedModel.generate's MLP on the host (model.py:680-685), eval mode: SN weights
    W / (u . W v) (spectral_norm.py:87-89), three Linear layers, LayerNormalization with the
    unbiased std (submodule.py:68-77)."""
    import torch.nn.functional as F
    x = torch.cat([noise, cls], 1)
    for L in (gen.generate_fc_layer, gen.des_rel_map_layer1, gen.des_rel_map_layer2):
        W = L.weight_orig.detach().cpu()
        sigma = torch.dot(L.weight_u.cpu(), torch.mv(W, L.weight_v.cpu()))
        x = F.linear(x, W / sigma, L.bias.detach().cpu())
    mu, sd = x.mean(-1, keepdim=True), x.std(-1, keepdim=True)
    return (x - mu.expand_as(x)) / (sd.expand_as(x) + gen.ln_eps) * gen.ln_a.detach().cpu() + gen.ln_b.detach().cpu()


def cpu_baseline_m3ae(enc, gen, w, budget_s: float = 15.0):
    """The reference's generate() on the host cores, relation by relation as ZSLmodule.eval calls
    it (zsl_module.py:662-667): test_sample rows of the 320-token description through the M3AE
    encoder over the full padded sequence (oracle/m3ae_text.py, torch CPU fp32) + the generator
    MLP, until the time budget."""
    import m3ae_text as om
    sd = {k: v.detach().cpu() for k, v in enc.state_dict().items()}
    S = w["test_sample"]
    g = torch.Generator().manual_seed(0)
    rows, r = 0, 0
    t0 = time.perf_counter()
    with torch.no_grad():
        while r < w["tok"].shape[0] and time.perf_counter() - t0 < budget_s:
            tok = w["tok"][r:r + 1].repeat(S, 1)
            msk = w["mask"][r:r + 1].repeat(S, 1)
            cls, _ = om.forward_representation_text(sd, tok, msk, enc.num_heads)
            _generator_cpu(gen, cls[:, 0], 0.1 * torch.randn(S, 15, generator=g))
            rows += S
            r += 1
    el = time.perf_counter() - t0
    return {"value": rows / el, "unit": "relation embeddings/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"first {r} FB15K-237-ZS relation descriptions x {S} rows ({rows} rows of 320 tokens) through "
                      f"M3AE-small forward_representation over the padded rows + generator MLP (oracle/m3ae_text.py, "
                      f"torch {torch.__version__} CPU fp32), {el:.2f} s on {torch.get_num_threads()} threads"}


def bench_m3ae(args, world, rank, dev, dist):
    """One step = UnifiedModel.generate (model.py:674-686) for every FB15K-237-ZS relation
    description x test_sample 20 (the ZSLmodule.eval expansion, zsl_module.py:662-666): 4,700
    description rows of 320 tokens -> row dedupe + padding-free HIP M3AE-small encoder -> CLS
    (N, 384) -> SN generator + LayerNormalization (HIP) -> (N, 200), D2H. N > 1: descriptions
    round-robin over ranks (independent rows, no collective)."""
    from mmre._lib import call, lib, ptr, stream_ptr
    from mmre.generator import RelationGenerator
    _lib_m3ae_plan_size = lib().mmre_m3ae_plan_size
    from mmre.m3ae import M3AETextEncoder
    from mmre.workloads import description_workload
    w = description_workload()
    R = int(w["tok"].shape[0])
    S = w["test_sample"]
    mine = np.arange(rank, R, world)
    torch.manual_seed(0)
    enc = M3AETextEncoder(w["vocab"], model_type="small").to(dev)
    gen = RelationGenerator(384, 15, 200).to(dev).eval()
    tok = w["tok"][mine].repeat_interleave(S, 0).to(dev)
    msk = w["mask"][mine].repeat_interleave(S, 0).to(dev)
    n = int(tok.shape[0])
    noise = 0.1 * torch.randn(n, 15, device=dev)
    host = torch.empty((n, 200), pin_memory=True)

    def step():
        with torch.no_grad():
            out = gen(enc.encode(tok, msk), noise)
        host.copy_(out, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=_coll_dev(dist, dev))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # roofline: the dominant kernel, fc1 (+GELU) of a block over the packed rows, timed alone
    plan = torch.empty(int(_lib_m3ae_plan_size(n)), dtype=torch.int32, device=dev)
    call("mmre_m3ae_plan", ptr(tok), ptr(msk), n, int(tok.shape[1]), 1, w["vocab"], ptr(plan), stream_ptr(dev))
    n_unique, packed = (int(v) for v in plan[3 * n + 1:3 * n + 3].cpu())
    d, hid = enc.emb_dim, 4 * enc.emb_dim
    A = torch.randn(packed, d, device=dev)
    fc1 = enc.encoder.blocks[0].transformer_mlp.fc1
    Hout = torch.empty(packed, hid, device=dev)
    st = stream_ptr(dev)
    launch = lambda: call("mmre_m3ae_linear", 1, ptr(A), packed, d, ptr(fc1.weight), hid, ptr(fc1.bias), None,
                          ptr(Hout), st)
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    k_ms = e0.elapsed_time(e1) / reps
    flops = 2.0 * packed * d * hid
    ach = flops / (k_ms * 1e-3) / 1e12
    if rank == 0:
        out = {"metric": f"relation embeddings generated/sec, {CONFIGS['m3ae']['workload']}",
               "value": R * S * args.steps / elapsed, "unit": "relation embeddings/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": "real FB15K-237-ZS relation-description lengths (synthetic token ids: no BERT vocabulary "
                       "offline), random-init M3AE-small encoder and generator",
               "config": {"workload": CONFIGS["m3ae"]["workload"], "descriptions": R, "rows": R * S,
                          "tokens_per_row": int(w["tok"].shape[1]), "unique_descriptions_rank0": n_unique,
                          "packed_rows_rank0": packed,
                          "parallelism": f"descriptions round-robin x{world}, no collective"},
               "roofline": {"bound": "mfma", "achieved": ach, "peak": MFMA_F32_PEAK / 1e12, "unit": "TFLOP/s",
                            "frac": ach * 1e12 / MFMA_F32_PEAK, "traffic": None,
                            "kernel": "k_m3ae_linear<1>", "kernel_ms": k_ms, "shape": [packed, d, hid],
                            "flops_per_launch": flops,
                            "note": "fc1+GELU of one block over the packed (unpadded) rows of the unique "
                                    "descriptions; the reference's padded rows and repeated descriptions are "
                                    "never computed"}}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_m3ae(enc, gen, w)
        print(json.dumps(_with_build(out)), flush=True)
    if dist:
        dist.destroy_process_group()


def rank_breakdown(ev, dist, dev, sweep_ms, n_local, entity_sharded, reps=20, fixed_ms=None):
    """Where an N > 1 evaluation's time goes, measured on EVERY rank after the timed region and
    all-gathered: the rank's local evaluation (entity / query prep, truth + filter kernels,
    sweep; a graph replay unless --eager), its sweep kernel alone, the fixed per-rank cost
    (fixed_ms: the eager twins' whole-call time minus their sweep, both from the same runs; with
    --eager, local - sweep), and the collective alone (the all-gather of the count lists with its
    scatter into query order, or the entity-sharded all-reduce), each the median of `reps`
    runs timed with events on the launch stream (barrier before every collective). Returns
    {name: [per-rank values]} and {name_min / name_max}."""
    from mmre.sharding import gather_counts, reduce_counts
    med = lambda xs: float(np.median(xs)) if xs else 0.0
    torch.cuda.synchronize()
    ev_pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    local = None
    for a, b in ev_pairs:
        a.record()
        local = ev._local()
        b.record()
    torch.cuda.synchronize()
    local_ms = med([a.elapsed_time(b) for a, b in ev_pairs])
    coll = []
    for a, b in ev_pairs:
        dist.barrier()
        torch.cuda.synchronize()
        a.record()
        if entity_sharded:
            reduce_counts(local.clone(), ev.group)
        else:
            gather_counts(local, ev.plan, ev.group)
        b.record()
        torch.cuda.synchronize()
        coll.append(a.elapsed_time(b))
    fixed = fixed_ms if fixed_ms is not None else max(local_ms - sweep_ms, 0.0)
    mine = torch.tensor([local_ms, sweep_ms, fixed, med(coll), float(n_local)],
                        dtype=torch.float64, device=_coll_dev(dist, dev))
    allv = torch.empty(dist.get_world_size() * 5, dtype=torch.float64, device=mine.device)  # flat: gloo's rule
    dist.all_gather_into_tensor(allv, mine)
    allv = allv.view(-1, 5).cpu().numpy()
    names = ["local_ms", "sweep_ms", "fixed_ms", "collective_ms", "sweeps"]
    per = {k: [round(float(x), 5) for x in allv[:, i]] for i, k in enumerate(names)}
    summ = {}
    for k in names:
        summ[k + "_min"] = float(allv[:, names.index(k)].min())
        summ[k + "_max"] = float(allv[:, names.index(k)].max())
    return per, summ


def _with_build(out):
    """Name the binary that produced the line (path, size, sha256 prefix of libmmre_hip.so)."""
    from mmre._lib import lib_identity
    out["build"] = lib_identity()
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict):
        cb.setdefault("cpu_model", _cpu_model())
        cb.setdefault("cores_note", _cores_note(int(cb.get("cores", 0))))
    return out


def _cores_note(used: int) -> str:
    """Why the CPU baseline ran on `used` threads (SURVEY 8(d) asks for the host's cores): the
    GPU pool gives each GPU's process a share of the host -- OMP_NUM_THREADS / MAX_JOBS are set
    to it (16 for one GPU of an 8-GPU node) -- while sched_getaffinity still lists every CPU of
    the machine, which the other GPUs' processes share. The baseline uses the share: torch's
    intra-op threads (= OMP_NUM_THREADS) for the reference's predict and as Base.so's
    workThreads."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 0
    omp = os.environ.get("OMP_NUM_THREADS")
    return (f"{used} threads = this process's CPU share (OMP_NUM_THREADS={omp}, torch intra-op threads "
            f"{torch.get_num_threads()}); sched_getaffinity lists {avail} CPUs, the whole host, shared with the other "
            f"GPUs' processes")


def _cpu_model():
    """The host CPU's model string (/proc/cpuinfo 'model name', what lscpu prints) and the
    number of CPUs this process may run on, so a cpu_baseline names the cores it ran on."""
    name = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count()
    return f"{name or 'unknown'} ({avail} CPUs available to the process)"


def _coll_dev(dist, dev):
    """Device for a small collective operand: the GPU under RCCL, the host under gloo."""
    return dev if dist.get_backend() == "nccl" else torch.device("cpu")


def _kfd_gpu_count() -> int:
    """GPUs of this node from the KFD topology (/sys/class/kfd/kfd/topology/nodes/*/properties:
    nodes with SIMDs), without any HIP call -- torch.cuda.device_count() may fall back to
    hipGetDeviceCount, which initialises HIP in the parent before the ranks are spawned. Honours
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES when set."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    props = dict(line.split(None, 1) for line in f if line.strip() and len(line.split()) == 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return 0
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        vis = os.environ.get(var)
        if vis is not None:
            n = min(n, len([x for x in vis.split(",") if x.strip()]))
    return n


def _self_launch(n: int) -> int:
    """`python bench.py --gpus N` (N > 1) without WORLD_SIZE: run this same command as N ranks of
    one torch.distributed.run job (one process per GPU, rendezvous on 127.0.0.1, a free port) and
    return its exit code. Called before any GPU call (the GPU count comes from the KFD topology,
    not from HIP; a HIP context already open here is refused); exits non-zero when the node has fewer than N GPUs, unless the gloo
    rehearsal (MMRE_BENCH_GLOO=1: every rank on cuda:0) was asked for."""
    import socket
    import subprocess
    have = _kfd_gpu_count()
    if torch.cuda.is_initialized():  # must not happen: the children would start under a live HIP context
        print("bench.py: HIP initialised before the self-launch; not measuring", file=sys.stderr)
        return 2
    if have < n and os.environ.get("MMRE_BENCH_GLOO") != "1":
        print(f"bench.py: --gpus {n} but this node has {have} GPU(s); not measuring", file=sys.stderr)
        return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="test triples in the CPU-baseline / parity sample (0: per-config default)")
    ap.add_argument("--train-steps", type=int, default=300,
                    help="HIP training steps that give the TransE configs non-degenerate tables (0: init tables)")
    ap.add_argument("--ns-neg", type=int, default=25, help="--config ns: negatives per positive (25 or 10)")
    ap.add_argument("--ns-eager", action="store_true", help="--config ns: launch each step eagerly (no hipGraph)")
    ap.add_argument("--ns-autograd", action="store_true",
                    help="--config ns (TransE): the drop-in path (sampler.sample + fused_ns_loss + backward + "
                         "SGD.step) instead of the one-call training step mmre_ns_step_openke")
    ap.add_argument("--ns-model", default="transe", choices=["transe", "distmult", "complex", "rotate"],
                    help="--config ns: the scored model (default transe, the C2 training step)")
    ap.add_argument("--ns-prefetch", action="store_true",
                    help="--config ns: sample the next batch on a forked stream while the current one trains "
                         "(default: in line before each step; the fork/join graph measured slower)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--init-tables", action="store_true",
                    help="C3/C4/C5: OpenKE-initialised tables (truths rank ~E/2) instead of structured ones")
    ap.add_argument("--eager", action="store_true",
                    help="link configs: launch each rank's local evaluation eagerly (default: one hipGraph replay)")
    ap.add_argument("--eval-streams", type=int, default=2, choices=[1, 2],
                    help="link configs: evaluation slots on separate HIP streams (2: evaluation i + 1's prep / "
                         "quantization / filter kernels run beside evaluation i's sweep; every evaluation does all "
                         "of its work)")
    ap.add_argument("--pack", default="cost", choices=["cost", "count"],
                    help="N > 1 relation-sharded: LPT by per-query cost (one calibration evaluation counts the pairs "
                         "the L1 filter leaves undecided; TransE) or by query count")
    ap.add_argument("--type-constrain", action="store_true",
                    help="link configs: the type-constrained evaluation (Tester.run_link_prediction(type_constrain=True), "
                         "Test.h:70-98 / 114-126) with type_constrain.txt built from the filter set as the reference's "
                         "n-n.py does (each relation's known heads / tails); metrics = the filter_tc group")
    ap.add_argument("--shard", default="relation", choices=["relation", "entity"],
                    help="N > 1 link configs: split the queries (relation-sharded, one all-gather; default) or "
                         "the entity table (every query against 1/N of the entities, one all-reduce)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around this process: start the N ranks here, as fresh children under
        # torch.distributed.run, before anything touches the GPU -- never a silent one-GPU run
        sys.exit(_self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to measure a different GPU count",
              file=sys.stderr)
        sys.exit(2)

    from mmre.link import FilterIndex, ScoreSpec, rotate_phase_denom
    from mmre.sharding import EntityShardedLinkEvaluation, ShardedLinkEvaluation
    from mmre.workloads import structured_tables, synthetic_large, train_transe, zs_workload
    # MMRE_BENCH_GLOO=1 rehearses the N > 1 path on a one-GPU box: every rank on cuda:0, gloo
    # collectives through host tensors (the driver's multi-GPU runs use RCCL, one rank per GPU)
    rehearse = world > 1 and os.environ.get("MMRE_BENCH_GLOO") == "1"
    dev_index = 0 if rehearse else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    dist = None
    # MMRE_BENCH_DIST=1 runs the collective path at world 1 too (RCCL init, barriers, the
    # one-rank all-gather / all-reduce): the RCCL code path checked on a one-GPU box
    if world > 1 or os.environ.get("MMRE_BENCH_DIST") == "1":
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    cfg = CONFIGS[args.config]
    if args.config == "zsl":
        return bench_zsl(args, world, rank, dev, dist)
    if args.config == "gan":
        return bench_gan(args, world, rank, dev, dist)
    if args.config == "ns":
        return bench_ns(args, world, rank, dev, dist)
    if args.config == "m3ae":
        return bench_m3ae(args, world, rank, dev, dist)
    if cfg["dataset"] == "synthetic-1M":
        w = synthetic_large(generator_device=dev)
    else:
        w = zs_workload(cfg["dataset"], cfg["model"], cfg["dim"], n_test=cfg.get("n_test"))
    if cfg["model"] != "transe" and not args.init_tables:
        # structured tables (truths near the top) so that the hit@k parity is not vacuous; C5 keeps
        # the generator's relation rows and pulls the entity rows toward them
        structured_tables(w, keep_rel=cfg["dataset"] == "synthetic-1M")
    w["norm_flag"] = cfg["norm"]
    model, dim = cfg["model"], cfg["dim"]
    if model == "transe" and args.train_steps > 0:
        train_transe(w, dev, steps=args.train_steps)
        if dist:  # every rank evaluates rank 0's tables (training is deterministic; one copy keeps it explicit)
            for k in ("ent", "rel"):
                t = w[k].to(_coll_dev(dist, dev))
                dist.broadcast(t, 0)
                w[k] = t.cpu()
    E = w["n_ent"]
    n = len(w["test_h"])
    tc = bool(args.type_constrain)
    if tc:  # type_constrain.txt by n-n.py's rule: each relation's known heads / tails (train + test)
        fh, fr, ft = (np.asarray(w[k], np.int64) for k in ("filter_h", "filter_r", "filter_t"))
        w["type_heads"] = [np.unique(fh[fr == r]) for r in range(w["n_rel"])]
        w["type_tails"] = [np.unique(ft[fr == r]) for r in range(w["n_rel"])]
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], E, w["n_rel"],
                        type_heads=w.get("type_heads"), type_tails=w.get("type_tails"))
    pk = {"transe": 0, "distmult": 2, "complex": 2, "rotate": 3}[model]
    spec = ScoreSpec(model=model, ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=dim,
                     ent_im=w.get("ent_im").to(dev) if "ent_im" in w else None,
                     rel_im=w.get("rel_im").to(dev) if "rel_im" in w else None, norm_flag=cfg["norm"],
                     pred_kind=pk, margin=float(w.get("margin", 0.0)),
                     phase_denom=rotate_phase_denom(w["margin"], w["epsilon"], dim) if model == "rotate" else 0.0)
    if args.shard == "entity":
        ev = EntityShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev,
                                         type_constrain=tc)
        n_local = 2 * n if ev.entity_range[1] > ev.entity_range[0] else 0
        e_local = ev.entity_range[1] - ev.entity_range[0]
    else:
        # the rank's local evaluation (entity / query prep, truth and filter kernels, sweep)
        # replayed from one hipGraph; kernel_ms comes from an eager twin after the timed region
        ev = ShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev,
                                   graph=not args.eager, cost="undecided" if args.pack == "cost" else None,
                                   streams=args.eval_streams, type_constrain=tc)
        n_local = int(ev.masks[rank].sum())
        e_local = E

    def steps(k, evs=None):
        # evaluation i + 1 is enqueued before the host reduces evaluation i's metrics, so that
        # reduction overlaps the next sweep; every evaluation's metrics are reduced in the loop
        metrics, pending = None, None
        for i in range(k):
            ticket = ev.launch(evs[i] if evs else None)
            if pending is not None:
                metrics = ev.finish(pending, copy_counts=False)[0]
            pending = ticket
        if pending is not None:
            metrics = ev.finish(pending, copy_counts=False)[0]
        return metrics

    steps(args.warmup)
    torch.cuda.synchronize()

    graphed = getattr(ev, "_graph_wanted", False)
    evs = None if graphed else [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                                for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    metrics = steps(args.steps, evs)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    fixed_ms = None
    if graphed and n_local:  # the sweep kernel alone: events on the launch stream of eager evaluations
        from mmre.link import LinkSweep
        sw = LinkSweep(spec)
        bufs = sw.alloc_queries(len(ev.q_host[0]))
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        # each eager twin also bracketed whole: its fixed cost (local - sweep) from the same run
        outer = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for e2, o2 in zip(evs, outer):
            o2[0].record()
            sw.run(*ev.q, filt=ev.filt, type_masks=ev.masks_tc, buffers=bufs, sweep_events=e2)
            o2[1].record()
        torch.cuda.synchronize()
        fixed_ms = float(np.median([o[0].elapsed_time(o[1]) - e[0].elapsed_time(e[1]) for o, e in zip(outer, evs)]))
        twin_fst = sw.filter_stats(bufs)
        print(f"eager twin filter record: {twin_fst}", file=sys.stderr)
        del sw, bufs
    sweep_ms = float(np.mean([a.elapsed_time(b) for a, b in evs])) if n_local else 0.0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=_coll_dev(dist, dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    _, counts = ev.run()  # one more evaluation outside the timed region: the counts the parity check reads
    fst = ev.filter_stats() if hasattr(ev, "filter_stats") else None  # the count-only filter's record (l1q / bf3)
    print(f"evaluation filter record: {fst}", file=sys.stderr)
    breakdown = None
    if world > 1:  # every rank's local / sweep / fixed / collective time, gathered (all ranks take part)
        breakdown = rank_breakdown(ev, dist, dev, sweep_ms, n_local, args.shard == "entity", fixed_ms=fixed_ms)

    total_triples = 2 * n * E
    value = total_triples * args.steps / elapsed
    if rank == 0:
        bpt = bytes_per_triple(model, dim)
        triples_launch = n_local * e_local
        # the sweep's time per evaluation for the roof: the eager twin's kernel time, but never more
        # than the measured step -- with two evaluation streams consecutive sweeps overlap (one's
        # ramp beside the other's tail), so a single sweep's latency can exceed the per-evaluation
        # time the pipeline achieves (C1 r5: 0.091 vs 0.080 ms); the step bounds the sweep's
        # throughput time from above, so the frac stays conservative
        step_ms = elapsed / args.steps * 1e3
        eff_ms = min(sweep_ms, step_ms) if sweep_ms > 0 else 0.0
        tps = triples_launch / (eff_ms * 1e-3) if eff_ms > 0 else 0.0
        # the TransE sweep kernel that counted: the probe's code width (8 / 16) or the f32 fallback
        l1_bits = fst.get("bits") if fst is not None and fst["kind"] == "l1q" else None
        if model == "transe" and l1_bits == 16:
            KERNEL_NAMES["transe"] = "k_sweep_valu<5, false, false, 0,"
        elif model == "transe" and fst is not None and fst["kind"] == "l1q" and l1_bits is None:
            KERNEL_NAMES["transe"] = "k_sweep_valu<0, false, false, 0,"
        if tc and model == "transe":  # the type-constrained variant of the same sweep
            KERNEL_NAMES["transe"] = KERNEL_NAMES["transe"].replace(", false, false,", ", true, false,")
        if model in ("distmult", "complex") and MFMA_FILTER:
            # the wide split-bf16 sweep (k_sweep_bf3w) runs where the split planes exceed 64 MB (C5),
            # as mmre_link_sweep_bf3 decides; MMRE_BF3_WIDE forces either
            k_tot = dim * (2 if model == "complex" else 1)
            e_pad = -(-e_local // 128) * 128
            wide_env = os.environ.get("MMRE_BF3_WIDE")
            wide = wide_env != "0" if wide_env is not None else e_pad * k_tot * 4 > 64 * 2 ** 20
            KERNEL_NAMES[model] = "k_sweep_bf3w<2," if wide else "k_sweep_bf3<2>"
        # (type-constrained lines: profiles/pmc_<config>_tc.json, the TC sweep variant's counters)
        pmc_cfg = args.config + ("_tc" if args.type_constrain else "")
        traffic, tsrc = pmc_traffic(pmc_cfg, model) if world == 1 else (None, None)
        if model in ("distmult", "complex") and fst is not None and fst["kind"] == "bf3" and not fst["fallback"]:
            # the split-bf16 filter: three bf16 products of K = dim x planes per triple on the bf16
            # MFMA (kernel_ms brackets the whole filtered sweep: split, sweep, rescoring)
            flops = 2.0 * dim * (2 if model == "complex" else 1)
            ach = tps * 3.0 * flops / 1e12
            roof = {"bound": "mfma", "achieved": ach, "peak": MFMA_BF16_PEAK / 1e12, "unit": "TFLOP/s (bf16 MFMA)",
                    "frac": ach * 1e12 / MFMA_BF16_PEAK, "flops_per_triple": 3.0 * flops,
                    "f32_equiv_TFLOPs": tps * flops / 1e12,
                    "f32_equiv_frac": tps * flops / MFMA_F32_PEAK,
                    "mfma_note": "executed flops = 3 bf16 products (hi.hi, hi.lo, lo.hi) x 2K per triple against the "
                                 "dense bf16 MFMA peak; f32_equiv = the triple's 2K algorithmic flops against the f32 "
                                 "MFMA peak (the exact sweep's roof, which the filter passes)"}
        elif model in ("distmult", "complex"):
            flops = 2.0 * dim * (2 if model == "complex" else 1)
            ach = tps * flops / 1e12
            roof = {"bound": "mfma", "achieved": ach, "peak": MFMA_F32_PEAK / 1e12, "unit": "TFLOP/s",
                    "frac": ach * 1e12 / MFMA_F32_PEAK, "flops_per_triple": flops}
        else:
            ops = valu_ops_per_triple(model, dim, l1_bits)
            ach = tps * ops / 1e12
            roof = {"bound": "valu", "achieved": ach, "peak": VALU_LANE_OPS / 1e12,
                    "unit": "TOP/s (VALU lane-ops: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz)",
                    "frac": ach * 1e12 / VALU_LANE_OPS, "valu_ops_per_triple": ops}
        roof.update({
            "traffic": traffic, "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, 2 x FETCH_SIZE + WRITE_SIZE)",
            "traffic_source": tsrc, "kernel": KERNEL_NAMES[model], "kernel_ms": sweep_ms,
            "kernel_ms_effective": eff_ms,
            "kernel_ms_note": "achieved uses kernel_ms_effective = min(kernel_ms (eager twin, events on its launch "
                              "stream), ms_per_step): overlapping evaluations on two streams can make one sweep's "
                              "latency exceed the per-evaluation time the pipeline achieves",
            "triples_per_launch": triples_launch, "bytes_per_triple": bpt,
            "hbm_algorithmic_x": tps * bpt / (HBM_PEAK_GBS * 1e9),
            "hbm_measured_GBs": (traffic / (eff_ms * 1e-3) / 1e9) if traffic and eff_ms else None,
            "note": "binding roof: VALU for TransE/RotatE (TransE: the integer filter's v_sad_u8, four elements per "
                    "half-rate instruction = 1/2 slot per element -- the 16-bit codes' v_sad_u16 when the probe picks them: "
                    "1 slot --, MMRE_L1_FILTER=0: sub + add-with-abs; RotatE: sub, sub, mul, "
                    "fma, add + v_sqrt_f32 at 4 slots, the fast filter's loop), f32 MFMA for "
                    "DistMult/ComplEx. hbm_algorithmic_x = SURVEY 8(d) algorithmic bytes (one entity row per "
                    "scored triple) / 8 TB/s: > 1 because each entity row is reused across a 128-query LDS tile; "
                    "the measured HBM traffic is in traffic / hbm_measured_GBs"})
        data = {"c1": "synthetic TransE tables trained on the FB15K-237-ZS test triples",
                "c2": "synthetic TransE tables trained on the FB15K-237-ZS test triples",
                "c5": "synthetic 1M-entity DistMult table; relation table = the zsl_module generator (random-init "
                      "UnifiedModel SN layers + LayerNormalization, HIP) over synthetic 384-d text CLS rows + noise; "
                      "4,096 random test triples (= the filter set)"}.get(args.config, f"synthetic {model} tables")
        if "tables" in w:
            data += (" -- structured tables (mmre.workloads.structured_tables: each test triple pulls its tail "
                     "toward the model's image of its head, so truths rank near the top)")
        elif "trained" not in w:
            data += " (OpenKE init, seed 0)"
        if args.config != "c5":
            data += (f" ({args.train_steps} steps of this build's HIP trainer: bit-exact OpenKE sampler + fused margin"
                     f" loss, SGD 1.0, margin 5, neg 25)" if "trained" in w else "") + \
                f" over the real {w['dataset']} test triples; filter set = all test triples + 272,115 synthetic train"
        coll = "RCCL" if not dist or dist.get_backend() == "nccl" else "gloo rehearsal (every rank on cuda:0)"
        metric = METRIC if args.config == "c2" else f"scored triples/sec, {cfg['workload']}"
        if tc:
            metric += " (type-constrained: Tester.run_link_prediction(type_constrain=True))"
        grp = "filter_tc" if tc else "filter"
        out = {"metric": metric,
               "value": value, "unit": "scored triples/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": data,
               "config": {"workload": cfg["workload"], "n_entities": E, "dim": dim, "n_sweeps": 2 * n,
                          "parallelism": (f"entity-sharded x{world} (1/N of the entity tiles per rank), {coll} all-reduce "
                                          f"of the count table" if args.shard == "entity" else
                                          f"query-sharded x{world} (relation-major LPT with relation splits"
                                          f"{', packed by calibrated per-query cost' if getattr(ev, 'weights', None) is not None else ''}"
                                          f"), {coll} all-gather of rank counts"),
                          "launch": ("hipGraph replay of each rank's local evaluation" if graphed else "eager") +
                                    (", two evaluation slots on two HIP streams (consecutive evaluations overlap)"
                                     if getattr(ev, "_streams", None) else "")},
               "roofline": roof,
               "metrics": {"group": grp, "hit10": metrics[grp]["hit10"], "hit3": metrics[grp]["hit3"],
                           "hit1": metrics[grp]["hit1"], "mrr": metrics[grp]["mrr"], "mr": metrics[grp]["mr"]},
               "parity": None}
        if tc:
            out["data"] += ("; type_constrain.txt built from the filter set by the reference n-n.py's rule (each "
                            "relation's known heads / tails)")
        if fst is not None and fst["kind"] == "l1q":
            pairs = int(n_local) * int(e_local)
            out["l1_filter"] = {"undecided_pairs": fst["undecided"],
                                "undecided_frac": fst["undecided"] / pairs if pairs else None,
                                "fallback_to_f32": fst["fallback"],
                                "code_bits": fst.get("bits"),
                                "note": "pairs the code bound (8- or 16-bit codes, code_bits: the device-side probe's "
                                        "choice) left undecided, each rescored with the canonical f32 chain "
                                        "(mmre_link_l1q_stats, rank 0's last evaluation); fallback_to_f32 = the "
                                        "quantization pass found M > 128 x mean|x| and the sweep ran the f32 path"}
        elif fst is not None and fst["kind"] == "bf3":
            pairs = int(n_local) * int(e_local)
            out["mfma_filter"] = {"undecided_pairs": fst["undecided"],
                                  "undecided_frac": fst["undecided"] / pairs if pairs else None,
                                  "fallback_to_f32": fst["fallback"],
                                  "note": "pairs the split-bf16 bound left undecided (truths included), each rescored "
                                          "with the canonical f32 chain (mmre_link_bf3_stats, rank 0's last "
                                          "evaluation); fallback_to_f32 = the pair list overflowed and the exact f32 "
                                          "MFMA sweep counted"}
        if "trained" in w:
            out["config"]["tables"] = w["trained"]
        elif "tables" in w:
            out["config"]["tables"] = w["tables"]
        if breakdown is not None:
            out["per_rank"], out["per_rank_summary"] = breakdown
            out["per_rank_note"] = ("medians of 20 runs per rank after the timed region: local_ms = the rank's local "
                                    "evaluation (prep, truth + filter, sweep), sweep_ms = its sweep kernel, fixed_ms = "
                                    "the eager twin's whole evaluation minus its sweep kernel (both timed in the same "
                                    "runs), collective_ms = the count exchange alone (barrier before each); "
                                    "roofline.kernel_ms is rank 0's sweep")
        if world > 1:
            # the sharded evaluation's gathered counts vs one-GPU evaluation of every query on
            # rank 0 (itself checked against the reference Base.so at N = 1): bit-equal counts
            # mean bit-equal hit@k at this GPU count
            from mmre.link import evaluate_link_prediction
            m1, (h1, t1) = evaluate_link_prediction(spec, w["test_h"], w["test_r"], w["test_t"], index=index,
                                                    type_constrain=tc)
            single = np.concatenate([h1, t1], 1)
            rows = 4 if tc else 2
            out["parity"] = {"source": f"{args.shard}-sharded x{world} gathered counts vs a one-GPU evaluation of all "
                                       f"{2 * n} sweeps on rank 0",
                             "sweeps": 2 * n, "counts_bit_equal": bool(np.array_equal(np.asarray(counts), single)),
                             "mismatched_sweeps": int((np.asarray(counts)[:rows] != single[:rows]).any(0).sum()),
                             "metrics_bit_equal": all(metrics[g][k] == m1[g][k] for g in
                                                      (("filter", "raw", "filter_tc", "raw_tc") if tc else
                                                       ("filter", "raw")) for k in m1[g])}
        if world == 1 and not args.no_cpu_baseline:
            ref = ref_tester_leg(w, args.cpu_sample or REF_SAMPLE[args.config])
            if ref is not None:
                out["cpu_baseline"] = cpu_baseline_block(ref, w)
                gs = sample_scores(spec, w, int(ref["n"]), dev)
                out["parity"] = parity_block(ref, counts, n, w, gs, tc=tc)
                del gs
        print(json.dumps(_with_build(out)), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
