"""ref_tester.py -- TEST INFRASTRUCTURE ONLY: the reference's CPU link-prediction path, run
as the bench's `cpu_baseline` leg and as the full-size parity checker of the GPU counts.

It is the OpenKE Tester loop (OpenKE/openke/config/Tester.py:70-91) on this host's cores:

    getHeadBatch (Test.h:36-43) -> model.predict on torch CPU -> testHead (Test.h:65-127)
    getTailBatch (Test.h:46-53) -> model.predict on torch CPU -> testTail (Test.h:130-192)
    test_link_prediction (Test.h:232-327) -> getTestLink{MRR,MR,Hit10,Hit3,Hit1}

with the reference's own ranker: ``oracle/_ref/Base.so``, compiled by ``oracle/Makefile``
from /root/reference/OpenKE/openke/base/Base.cpp (the checker, never the product). The
``predict_*`` functions below are the reference models' torch op sequences, unchanged in
order and dtype (TransE.py:46-74 + 88-94, DistMult.py:34-55 + 70-72, ComplEx.py:20-40 +
60-62, RotatE.py:45-91); ``tests/test_oracle_golden.py`` pins them bit-for-bit against the
reference's own predictions in tests/golden/link_small.npz.

Per query it also reads Base.so's rank deltas (l_rank / l_filter_rank / r_rank /
r_filter_rank are float globals holding sums of exact integers below 2^24), so the GPU's
per-query counts can be compared with the reference's one by one, and it returns the
reference's score vectors (model.predict output of every sweep), so the caller can measure
the GPU-vs-reference score error sweep by sweep and count the entities inside that error
window around the truth -- the only ones whose side of the strict `<` (Test.h:83, :147) a
different float summation order can flip. `near_ties` is a cruder, score-only screen
(entities within ``tie_rel`` x max|score| of the truth).

Usage (a child process of bench.py: Base.so is C++ with unguarded indexing):
    python oracle/ref_tester.py <workdir>
<workdir> holds the OpenKE files (entity2id / relation2id / train2id / valid2id / test2id),
tables.npz (ent, rel[, ent_im, rel_im]) and meta.json (model, dim, norm_flag, margin,
epsilon, threads[, summary, near_rel]); the result goes to <workdir>/result.npz. With
``summary`` the score vectors are not kept (C5's would be 8 MB per sweep): per sweep it keeps
the truth's reference score, max|s| and every other entity whose reference score lies within
near_rel x max|s| of the truth's (ids + scores, CSR) -- the only entities whose side of the
strict `<` a different summation order can flip (tests/golden/make_ref_parity.py).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_BASE_SO = os.path.join(HERE, "_ref", "Base.so")


# ----------------------------------------------------------- reference predict --
def predict_transe(ent, rel, ph, pt, pr, mode, norm_flag=True, p_norm=1, margin=None):
    """TransE.forward + predict (TransE.py:46-74, 88-94): gather, F.normalize(2, -1),
    view(-1, R, d), h + (r - t) for head_batch else (h + r) - t, torch.norm(p, -1);
    predict = margin - (margin - score) with a margin, the score otherwise."""
    import torch
    import torch.nn.functional as F
    h, t, r = ent[ph], ent[pt], rel[pr]
    if norm_flag:
        h = F.normalize(h, 2, -1)
        r = F.normalize(r, 2, -1)
        t = F.normalize(t, 2, -1)
    h = h.view(-1, r.shape[0], h.shape[-1])
    t = t.view(-1, r.shape[0], t.shape[-1])
    r = r.view(-1, r.shape[0], r.shape[-1])
    s = h + (r - t) if mode == "head_batch" else (h + r) - t
    score = torch.norm(s, p_norm, -1).flatten()
    if margin is not None:
        m = torch.tensor([margin], dtype=torch.float32)
        score = m - (m - score)  # forward returns margin - score (:70-71), predict margin - forward (:90-91)
    return score.cpu().data.numpy()


def predict_distmult(ent, rel, ph, pt, pr, mode):
    """DistMult._calc + predict (DistMult.py:34-55, 70-72)."""
    import torch
    h, t, r = ent[ph], ent[pt], rel[pr]
    h = h.view(-1, r.shape[0], h.shape[-1])
    t = t.view(-1, r.shape[0], t.shape[-1])
    r = r.view(-1, r.shape[0], r.shape[-1])
    s = h * (r * t) if mode == "head_batch" else (h * r) * t
    score = torch.sum(s, -1).flatten()
    return (-score).cpu().data.numpy()


def predict_complex(ent_re, ent_im, rel_re, rel_im, ph, pt, pr, mode):
    """ComplEx._calc + predict (ComplEx.py:20-40, 60-62): no mode handling, broadcast."""
    import torch
    h_re, h_im, t_re, t_im = ent_re[ph], ent_im[ph], ent_re[pt], ent_im[pt]
    r_re, r_im = rel_re[pr], rel_im[pr]
    score = torch.sum(h_re * t_re * r_re + h_im * t_im * r_re + h_re * t_im * r_im - h_im * t_re * r_im, -1)
    return (-score).cpu().data.numpy()


def predict_rotate(ent, rel, ph, pt, pr, mode, margin, epsilon, dim):
    """RotatE._calc + forward + predict (RotatE.py:45-91): phase = r / (range / pi),
    rotate, stack, norm(dim=0).sum(-1), forward = margin - score, predict = -forward."""
    import torch
    pi = 3.14159265358979323846
    rel_range = torch.tensor([(margin + epsilon) / dim], dtype=torch.float32)
    h, t, r = ent[ph], ent[pt], rel[pr]
    re_head, im_head = torch.chunk(h, 2, dim=-1)
    re_tail, im_tail = torch.chunk(t, 2, dim=-1)
    phase = r / (rel_range.item() / pi)
    re_rel, im_rel = torch.cos(phase), torch.sin(phase)
    R = re_rel.shape[0]
    re_head = re_head.view(-1, R, re_head.shape[-1]).permute(1, 0, 2)
    re_tail = re_tail.view(-1, R, re_tail.shape[-1]).permute(1, 0, 2)
    im_head = im_head.view(-1, R, im_head.shape[-1]).permute(1, 0, 2)
    im_tail = im_tail.view(-1, R, im_tail.shape[-1]).permute(1, 0, 2)
    im_rel = im_rel.view(-1, R, im_rel.shape[-1]).permute(1, 0, 2)
    re_rel = re_rel.view(-1, R, re_rel.shape[-1]).permute(1, 0, 2)
    if mode == "head_batch":
        re_s = re_rel * re_tail + im_rel * im_tail
        im_s = re_rel * im_tail - im_rel * re_tail
        re_s = re_s - re_head
        im_s = im_s - im_head
    else:
        re_s = re_head * re_rel - im_head * im_rel
        im_s = re_head * im_rel + im_head * re_rel
        re_s = re_s - re_tail
        im_s = im_s - im_tail
    score = torch.stack([re_s, im_s], dim=0).norm(dim=0).sum(dim=-1).permute(1, 0).flatten()
    m = torch.tensor([margin], dtype=torch.float32)
    return (-(m - score)).cpu().data.numpy()


def make_predict(meta, tables):
    """predict(ph, pt, pr, mode) -> float32 numpy for the model named in meta."""
    import torch
    T = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in tables.items()}
    model = meta["model"]
    if model in ("transe", "transe_l2"):
        p = 1 if model == "transe" else 2
        return lambda ph, pt, pr, mode: predict_transe(T["ent"], T["rel"], ph, pt, pr, mode,
                                                       norm_flag=meta.get("norm_flag", True), p_norm=p,
                                                       margin=meta.get("transe_margin"))
    if model == "distmult":
        return lambda ph, pt, pr, mode: predict_distmult(T["ent"], T["rel"], ph, pt, pr, mode)
    if model == "complex":
        return lambda ph, pt, pr, mode: predict_complex(T["ent"], T["ent_im"], T["rel"], T["rel_im"], ph, pt, pr,
                                                        mode)
    if model == "rotate":
        return lambda ph, pt, pr, mode: predict_rotate(T["ent"], T["rel"], ph, pt, pr, mode, meta["margin"],
                                                       meta["epsilon"], meta["dim"])
    raise ValueError(f"unknown model {model}")


# ------------------------------------------------------------------ Tester loop --
@contextlib.contextmanager
def stdout_to_stderr():
    """Base.so printf()s to fd 1."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _fglob(lib, name):
    return ctypes.c_float.in_dll(lib, name).value


def near_ties(scores, truth, tie_rel):
    """#{j != truth : |s_j - s_truth| <= tie_rel * max_j |s_j|} per sweep."""
    s = np.asarray(scores, np.float64)
    st = s[np.arange(s.shape[0]), truth][:, None]
    tol = tie_rel * np.max(np.abs(s), axis=1, keepdims=True)
    close = np.abs(s - st) <= tol
    close[np.arange(s.shape[0]), truth] = False
    return close.sum(1)


def prepare_workdir(workdir: str, w: dict, th, tr, tt, **meta_extra):
    """Write the OpenKE directory + tables + meta a Tester run over the sample (th, tr, tt)
    needs: test2id = the sample; train2id = the workload's filter set minus one copy of each
    sampled triple, so Base.so filters with exactly the triples the GPU evaluation filters
    with; one valid triple, a copy of a sampled test triple (already in the filter set):
    Reader.h:255-256 reads validList[0] unguarded, so an empty valid2id.txt crashes Base.so
    intermittently."""
    th, tr, tt = (np.asarray(x, np.int64) for x in (th, tr, tt))
    fh, fr, ft = (np.asarray(w[k], np.int64) for k in ("filter_h", "filter_r", "filter_t"))
    keep = np.ones(len(fh), bool)
    key = (fh * w["n_rel"] + fr) * w["n_ent"] + ft
    skey = (th * w["n_rel"] + tr) * w["n_ent"] + tt
    pos = {}
    for i, k in enumerate(key.tolist()):
        pos.setdefault(k, i)
    for k in skey.tolist():
        if k in pos:
            keep[pos.pop(k)] = False
    trn = np.stack([fh[keep], ft[keep], fr[keep]], 1)
    tst = np.stack([th, tt, tr], 1)
    for name, arr in (("train2id.txt", trn), ("valid2id.txt", tst[:1]), ("test2id.txt", tst)):
        with open(os.path.join(workdir, name), "w") as f:
            f.write(f"{len(arr)}\n")
            np.savetxt(f, arr, fmt="%d")
    for name, cnt in (("entity2id.txt", w["n_ent"]), ("relation2id.txt", w["n_rel"])):
        with open(os.path.join(workdir, name), "w") as f:
            f.write(f"{cnt}\n")
    if w.get("type_heads") is not None:
        # type_constrain.txt as importTypeFiles (Reader.h:267-317) reads it: the relation count,
        # then per relation (every one, in order) a head line and a tail line "r n e1 .. en"
        with open(os.path.join(workdir, "type_constrain.txt"), "w") as f:
            f.write(f"{w['n_rel']}\n")
            for r in range(int(w["n_rel"])):
                for lists in (w["type_heads"], w["type_tails"]):
                    ids = [int(x) for x in lists[r]]
                    f.write(f"{r}\t{len(ids)}" + "".join(f"\t{e}" for e in ids) + "\n")
        meta_extra = dict(meta_extra, type_constrain=True)
    as_np = lambda v: v.numpy() if hasattr(v, "numpy") else np.asarray(v)
    tables = {"ent": as_np(w["ent"]), "rel": as_np(w["rel"])}
    if "ent_im" in w:
        tables.update(ent_im=as_np(w["ent_im"]), rel_im=as_np(w["rel_im"]))
    np.savez(os.path.join(workdir, "tables.npz"), **tables)
    meta = dict(model=w["model"], dim=w["dim"], norm_flag=bool(w.get("norm_flag", False)),
                margin=w.get("margin"), epsilon=w.get("epsilon"))
    meta.update(meta_extra)
    with open(os.path.join(workdir, "meta.json"), "w") as f:
        json.dump(meta, f)


def run_tester(workdir: str, base_so: str = REF_BASE_SO, tie_rel: float = 1e-4):
    import torch
    with open(os.path.join(workdir, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("threads"):
        torch.set_num_threads(int(meta["threads"]))
    with np.load(os.path.join(workdir, "tables.npz"), allow_pickle=False) as z:
        tables = {k: z[k] for k in z.files}
    predict = make_predict(meta, tables)
    lib = ctypes.CDLL(base_so)
    P, I = ctypes.c_void_p, ctypes.c_int64
    lib.setInPath.argtypes = [ctypes.c_char_p]
    lib.getHeadBatch.argtypes = [P, P, P]
    lib.getTailBatch.argtypes = [P, P, P]
    lib.testHead.argtypes = [P, I, I]
    lib.testTail.argtypes = [P, I, I]
    lib.test_link_prediction.argtypes = [I]
    for g in ("getTestLinkMRR", "getTestLinkMR", "getTestLinkHit10", "getTestLinkHit3", "getTestLinkHit1"):
        getattr(lib, g).argtypes = [I]
        getattr(lib, g).restype = ctypes.c_float
    lib.getEntityTotal.restype = I
    lib.getTestTotal.restype = I
    tc = bool(meta.get("type_constrain", False))  # Test.h's type-constrained counters too
    with stdout_to_stderr():
        lib.setInPath((workdir.rstrip("/") + "/").encode())
        lib.importTrainFiles()
        lib.importTestFiles()
        if tc:
            lib.importTypeFiles()
        lib.initTest()
    E, n = int(lib.getEntityTotal()), int(lib.getTestTotal())
    ph, pt, pr = (np.zeros(E, np.int64) for _ in range(3))
    counts = np.zeros((2, n, 4 if tc else 2), np.int64)  # [head|tail][query][raw, filt(, raw_tc, filt_tc)]
    q = np.zeros((n, 3), np.int64)               # (h, r, t) as Base.so's testList holds them
    summary = bool(meta.get("summary", False))
    near_rel = float(meta.get("near_rel", 1e-5))
    scores = None if summary else np.zeros((2, n, E), np.float32)
    truth_s = np.zeros((2, n), np.float32)
    smax = np.zeros((2, n), np.float32)
    near_ids, near_cnt = [], np.zeros((2, n), np.int64)

    def keep(side, idx, s, truth):
        truth_s[side, idx] = s[truth]
        smax[side, idx] = np.max(np.abs(s))
        if scores is not None:
            scores[side, idx] = s
        else:
            tol = near_rel * float(smax[side, idx])
            j = np.flatnonzero(np.abs(s.astype(np.float64) - float(s[truth])) <= tol)
            j = j[j != truth]
            near_ids.append((side, idx, j.astype(np.int32), s[j]))
            near_cnt[side, idx] = len(j)

    keys = (("l_rank", "l_filter_rank"), ("r_rank", "r_filter_rank"))
    if tc:
        keys = tuple(k + (f"{s}_rank_constrain", f"{s}_filter_rank_constrain") for k, s in zip(keys, ("l", "r")))
    t_keep = 0.0
    t_idx = np.zeros(n, np.float64)  # per test triple (both sweeps), the fixture bookkeeping excluded
    t0 = time.perf_counter()
    with stdout_to_stderr():
        for idx in range(n):
            ti = time.perf_counter()
            lib.getHeadBatch(ph.ctypes.data, pt.ctypes.data, pr.ctypes.data)
            s = np.ascontiguousarray(predict(torch.from_numpy(ph), torch.from_numpy(pt[:1]),
                                             torch.from_numpy(pr[:1]), "head_batch"), np.float32)
            before = [_fglob(lib, k) for k in keys[0]]
            lib.testHead(s.ctypes.data, idx, int(tc))
            counts[0, idx] = [round(_fglob(lib, k) - b) - 1 for k, b in zip(keys[0], before)]
            q[idx, 1], q[idx, 2] = pr[0], pt[0]
            head_s = s
            lib.getTailBatch(ph.ctypes.data, pt.ctypes.data, pr.ctypes.data)
            s = np.ascontiguousarray(predict(torch.from_numpy(ph[:1]), torch.from_numpy(pt),
                                             torch.from_numpy(pr[:1]), "tail_batch"), np.float32)
            before = [_fglob(lib, k) for k in keys[1]]
            lib.testTail(s.ctypes.data, idx, int(tc))
            counts[1, idx] = [round(_fglob(lib, k) - b) - 1 for k, b in zip(keys[1], before)]
            q[idx, 0] = ph[0]
            k0 = time.perf_counter()
            t_idx[idx] = k0 - ti
            keep(0, idx, head_s, int(q[idx, 0]))   # the head sweep's truth is the tail batch's anchor
            keep(1, idx, s, int(q[idx, 2]))
            t_keep += time.perf_counter() - k0
        lib.test_link_prediction(int(tc))
        elapsed = time.perf_counter() - t0 - t_keep
        g = int(tc)  # getTestLink*(type_constrain): the type-constrained filtered metrics when tc
        metrics = np.array([lib.getTestLinkMRR(g), lib.getTestLinkMR(g), lib.getTestLinkHit10(g),
                            lib.getTestLinkHit3(g), lib.getTestLinkHit1(g)], np.float32)
    if not all(math.isfinite(float(m)) for m in metrics):
        raise RuntimeError("Base.so returned non-finite metrics")
    out = dict(counts=counts, q=q, metrics=metrics, elapsed=np.float64(elapsed), t_idx=t_idx,
               threads=np.int64(torch.get_num_threads()), n_ent=np.int64(E), tie_rel=np.float64(tie_rel),
               truth_scores=truth_s, score_absmax=smax)
    if scores is not None:
        out["scores"] = scores
        out["near_ties"] = np.stack([near_ties(scores[0], q[:, 0], tie_rel), near_ties(scores[1], q[:, 2], tie_rel)])
    else:
        # near lists in sweep order [head sweeps 0..n-1 | tail sweeps 0..n-1]
        near_ids.sort(key=lambda x: (x[0], x[1]))
        out["near_off"] = np.r_[0, np.cumsum(near_cnt.reshape(-1))].astype(np.int64)
        out["near_ids"] = (np.concatenate([x[2] for x in near_ids]) if near_ids else np.zeros(0, np.int32))
        out["near_scores"] = (np.concatenate([x[3] for x in near_ids]) if near_ids else np.zeros(0, np.float32))
        out["near_rel"] = np.float64(near_rel)
        out["near_ties"] = near_cnt
    np.savez(os.path.join(workdir, "result.npz"), **out)
    return out


def run_parallel(w: dict, th, tr, tt, procs: int, timeout_s: float | None = None, **meta_extra):
    """The Tester loop over the sample (th, tr, tt) -- kept in Test.h order -- cut into `procs`
    contiguous chunks, each a child process with its own Base.so on one torch thread (torch's
    intra-op threads do not speed the reference's predict up: 1.4 s per C4 triple on 1 thread,
    1.7 s on 8). Each chunk's train2id is the filter set minus its own test triples, so every
    child filters with the whole filter set, exactly as one run over the sample would.

    Merged result = run_tester's, over the whole sample: counts / q / truth_scores /
    score_absmax / near lists in the one-run order ([head sweeps | tail sweeps] for the CSR
    lists), elapsed = the slowest chunk's Tester loop (the chunks run side by side; startup
    and the near-list bookkeeping excluded), threads = the processes used. Base.so's metrics
    are per chunk; the sample's are the Test.h:232-327 reduction of the merged counts
    restated by the oracle (oracle.link_metrics), which must reproduce every chunk's Base.so
    metrics bit for bit first (kept as chunk_metrics)."""
    import shutil
    import subprocess
    import tempfile
    sys.path.insert(0, HERE)
    import oracle as orc
    th, tr, tt = (np.asarray(x, np.int64) for x in (th, tr, tt))
    n = len(th)
    procs = max(1, min(int(procs), n))
    bounds = np.linspace(0, n, procs + 1).round().astype(np.int64)
    tmps, kids = [], []
    try:
        for c in range(procs):
            a, b = int(bounds[c]), int(bounds[c + 1])
            tmp = tempfile.mkdtemp(prefix=f"mmre_refpar{c}_")
            tmps.append(tmp)
            prepare_workdir(tmp, w, th[a:b], tr[a:b], tt[a:b], threads=1, **meta_extra)
        env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
        for tmp in tmps:
            kids.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), tmp], stdout=subprocess.DEVNULL,
                                         stderr=subprocess.DEVNULL, env=env))
        t0 = time.time()
        for k in kids:
            left = None if timeout_s is None else max(1.0, timeout_s - (time.time() - t0))
            if k.wait(timeout=left) != 0:
                raise RuntimeError(f"ref_tester chunk failed rc={k.returncode}")
        parts = []
        for tmp in tmps:
            with np.load(os.path.join(tmp, "result.npz"), allow_pickle=False) as z:
                parts.append({k: z[k] for k in z.files})
    finally:
        for k in kids:
            if k.poll() is None:
                k.kill()
                k.wait()
        for tmp in tmps:
            shutil.rmtree(tmp, ignore_errors=True)

    def tc4(c):  # (2, m, 2) [raw, filt] (or (2, m, 4) with the type-constrained pair) -> the oracle's (m, 4)
        if c.shape[2] == 4:
            return [c[0], c[1]]
        z = np.zeros((c.shape[1], 4), np.int64)
        return [np.concatenate([c[s], z[:, :2]], 1) for s in (0, 1)]

    grp = "filter_tc" if parts[0]["counts"].shape[2] == 4 else "filter"
    for c, p in enumerate(parts):
        m = orc.link_metrics(*tc4(p["counts"]))[grp]
        mine = np.array([m[k] for k in orc.METRIC_NAMES], np.float32)
        if not np.array_equal(mine.view(np.uint32), p["metrics"].astype(np.float32).view(np.uint32)):
            raise RuntimeError(f"chunk {c}: the oracle's metric reduction {mine} differs from Base.so's {p['metrics']}")
    cat1 = lambda k: np.concatenate([p[k] for p in parts], axis=1)
    counts = cat1("counts")
    m = orc.link_metrics(*tc4(counts))[grp]
    out = dict(counts=counts, q=np.concatenate([p["q"] for p in parts]),
               metrics=np.array([m[k] for k in orc.METRIC_NAMES], np.float32),
               chunk_metrics=np.stack([p["metrics"] for p in parts]), chunk_n=np.diff(bounds),
               elapsed=np.float64(max(float(p["elapsed"]) for p in parts)),
               elapsed_chunks=np.array([float(p["elapsed"]) for p in parts]),
               t_idx=np.concatenate([p["t_idx"] for p in parts]), threads=np.int64(procs),
               n_ent=parts[0]["n_ent"], tie_rel=parts[0]["tie_rel"], truth_scores=cat1("truth_scores"),
               score_absmax=cat1("score_absmax"), near_ties=cat1("near_ties"))
    if "scores" in parts[0]:
        out["scores"] = cat1("scores")
    if "near_off" in parts[0]:
        ids, sc, cnt = [], [], []
        for side in (0, 1):
            for p in parts:
                nc, off = p["counts"].shape[1], p["near_off"]
                for i in range(side * nc, (side + 1) * nc):
                    ids.append(p["near_ids"][off[i]:off[i + 1]])
                    sc.append(p["near_scores"][off[i]:off[i + 1]])
                    cnt.append(off[i + 1] - off[i])
        out["near_off"] = np.r_[0, np.cumsum(cnt)].astype(np.int64)
        out["near_ids"] = np.concatenate(ids).astype(np.int32) if ids else np.zeros(0, np.int32)
        out["near_scores"] = np.concatenate(sc).astype(np.float32) if sc else np.zeros(0, np.float32)
        out["near_rel"] = parts[0]["near_rel"]
    return out


if __name__ == "__main__":
    r = run_tester(sys.argv[1])
    print(f"ref_tester: {r['counts'].shape[1]} test triples x 2 sweeps in {float(r['elapsed']):.2f} s "
          f"on {int(r['threads'])} threads")
