"""oracle.py -- TEST INFRASTRUCTURE ONLY: the parity oracle.

Python front-end of the CPU restatement of the reference's hot path. Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
import this module, and only as the checker; the product package never does.

* ``liboracle.so`` (``mmre_oracle.c``) restates the OpenKE scoring
  (``TransE.py:62-76``, ``DistMult.py:34-44``, ``ComplEx.py:20-27``,
  ``RotatE.py:45-76``), the Test.h ranker (``Test.h:65-192``, ``Corrupt.h:166-177``),
  the metric accumulation (``Test.h:232-327``), the Base.cpp sampler
  (``Base.cpp:78-197``, ``Corrupt.h:7-163``, ``Random.h:11-29``) and the
  ``main.evaluate`` candidate ranking (``main.py:232-250``).
* numpy restates the Reader.h training index (``Reader.h:53-160``), the
  generator MLP (``module/model.py:674-686``, ``module/spectral_norm.py:39-89``,
  ``module/submodule.py:58-77``) and the ZSL cosine ranking
  (``module/zsl_module.py:699-706``).

Pinned against tests/golden/*.npz (made by tests/golden/make_golden.py from the
reference itself in the build container).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_BASE_SO = os.path.join(HERE, "_ref", "Base.so")

MODELS = {"transe": 0, "transe_l2": 1, "distmult": 2, "complex": 3, "rotate": 4}
MODES = {"head_batch": 0, "tail_batch": 1}

_lib = None
_P = ctypes.c_void_p
_I = ctypes.c_int64


def build(ref: bool = False) -> None:
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    if ref and os.path.exists("/root/reference/OpenKE/openke/base/Base.cpp"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_link_predict.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                       _P, _P, _P, _P, _I, ctypes.c_int, ctypes.c_float, _P, _P, _P, _I, _P]
        L.orc_test_rank.argtypes = [ctypes.c_int, _P, _I, _P, _P, _P, _I, _P, _I, _P, _P, _P]
        L.orc_link_metrics.argtypes = [_P, _P, _I, _P]
        L.orc_glibc_rand.argtypes = [_I, _P]
        L.orc_sampling.argtypes = [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _I,
                                   _P, _P, _P, _P, _I, _I, _I, _I, _P]
        L.orc_import_prob.argtypes = [ctypes.c_char_p, _I, ctypes.c_float, _P]
        L.orc_candidate_rank_transe.argtypes = [_P, _P, ctypes.c_int, _P, _P, _P, _P, _I, _P, _P]
        L.orc_sincos_vec.argtypes = [_P, _I, _P, _P]
        L.orc_normalize_rows.argtypes = [_P, _I, ctypes.c_int, _P]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def _i64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.int64)


# ------------------------------------------------------------------ scoring --
def pred_kind(model: str, has_margin: bool) -> int:
    """Which transform model.predict applies to the raw score (see mmre_oracle.c header)."""
    if model in ("transe", "transe_l2"):
        return 1 if has_margin else 0
    if model in ("distmult", "complex"):
        return 2
    return 3


def rotate_phase_denom(margin: float, epsilon: float, dim: int) -> np.float32:
    """``rel_embedding_range.item() / pi`` (RotatE.py:31-34, 51): python float / f32 tensor is
    evaluated by torch as ``reciprocal(pi) * range`` in float32 (BaseModule.py:10 pi_const)."""
    rng = np.float32((margin + epsilon) / dim)
    pi = np.float32(3.14159265358979323846)
    return np.float32(np.float32(np.float32(1.0) / pi) * rng)


def link_predict(model, mode, ent, rel, qh, qr, qt, ent_im=None, rel_im=None, norm_flag=True,
                 margin=None, phase_denom=0.0):
    """(Q, E) predicted values as model.predict returns them for each query sweep."""
    ent, rel, ent_im, rel_im = _f32(ent), _f32(rel), _f32(ent_im), _f32(rel_im)
    qh, qr, qt = _i64(qh), _i64(qr), _i64(qt)
    E = ent.shape[0]
    d = rel.shape[1]
    Q = qh.shape[0]
    out = np.empty((Q, E), dtype=np.float32)
    pk = pred_kind(model, margin is not None)
    lib().orc_link_predict(MODELS[model], MODES[mode], int(bool(norm_flag)), pk,
                           float(margin or 0.0), _ptr(ent), _ptr(ent_im), _ptr(rel), _ptr(rel_im), E, d,
                           float(phase_denom), _ptr(qh), _ptr(qr), _ptr(qt), Q, _ptr(out))
    return out


def sincos(x):
    x = _f32(x)
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib().orc_sincos_vec(_ptr(x), x.size, _ptr(s), _ptr(c))
    return s, c


def normalize_rows(x):
    x = _f32(x)
    out = np.empty_like(x)
    lib().orc_normalize_rows(_ptr(x), x.shape[0], x.shape[1], _ptr(out))
    return out


# ------------------------------------------------------------------ ranking --
def sorted_hrt(h, r, t):
    """train+valid+test triples as unique (h, r, t) rows in cmp_head order (Reader.h:226)."""
    a = np.stack([np.asarray(h, np.int64), np.asarray(r, np.int64), np.asarray(t, np.int64)], 1)
    a = np.unique(a, axis=0)
    return np.ascontiguousarray(a)


def test_rank(mode, pred, qh, qr, qt, hrt_sorted, type_off=None, type_ids=None):
    """(Q, 4) int64: raw, filtered, raw-constrained, filtered-constrained (Test.h:65-192)."""
    pred = _f32(pred)
    qh, qr, qt = _i64(qh), _i64(qr), _i64(qt)
    hrt_sorted = _i64(hrt_sorted)
    out = np.zeros((qh.shape[0], 4), dtype=np.int64)
    lib().orc_test_rank(MODES[mode], _ptr(pred), pred.shape[1], _ptr(qh), _ptr(qr), _ptr(qt), qh.shape[0],
                        _ptr(hrt_sorted), hrt_sorted.shape[0], _ptr(_i64(type_off)), _ptr(_i64(type_ids)),
                        _ptr(out))
    return out


METRIC_NAMES = ["mrr", "mr", "hit10", "hit3", "hit1"]


def link_metrics(head_counts, tail_counts):
    """Test.h:232-327 (P14 float semantics). Returns dict of 4 groups x 5 floats."""
    h = _i64(head_counts)
    t = _i64(tail_counts)
    out = np.zeros(20, dtype=np.float32)
    lib().orc_link_metrics(_ptr(h), _ptr(t), h.shape[0], _ptr(out))
    res = {}
    for g, grp in enumerate(["filter", "raw", "filter_tc", "raw_tc"]):
        res[grp] = {n: np.float32(out[5 * g + i]) for i, n in enumerate(METRIC_NAMES)}
    return res


# ----------------------------------------------------------------- sampling --
def glibc_rand(n):
    out = np.zeros(n, dtype=np.int64)
    lib().orc_glibc_rand(n, _ptr(out))
    return out


def train_index(h, t, r, n_ent, n_rel):
    """Restates importTrainFiles (Reader.h:53-160) with numpy."""
    a = np.unique(np.stack([np.asarray(h), np.asarray(r), np.asarray(t)], 1).astype(np.int64), axis=0)
    train_list = a  # (h, r, t) in cmp_head order
    head = a
    tail = a[np.lexsort((a[:, 0], a[:, 1], a[:, 2]))]  # (t, r, h)
    rel = a[np.lexsort((a[:, 1], a[:, 2], a[:, 0]))]   # (h, t, r)

    def lefrig(keys):
        lef = np.zeros(n_ent, np.int64)
        rig = np.full(n_ent, -1, np.int64)
        idx = np.arange(keys.shape[0])
        first = np.ones(keys.shape[0], bool)
        first[1:] = keys[1:] != keys[:-1]
        last = np.ones(keys.shape[0], bool)
        last[:-1] = keys[1:] != keys[:-1]
        lef[keys[first]] = idx[first]
        rig[keys[last]] = idx[last]
        return lef, rig

    lef_head, rig_head = lefrig(head[:, 0])
    lef_tail, rig_tail = lefrig(tail[:, 2])
    lef_rel, rig_rel = lefrig(rel[:, 0])
    freq = np.bincount(a[:, 1], minlength=n_rel).astype(np.float32)
    hr = np.unique(a[:, :2], axis=0)
    tr = np.unique(a[:, [2, 1]], axis=0)
    left_cnt = np.bincount(hr[:, 1], minlength=n_rel).astype(np.float32)
    right_cnt = np.bincount(tr[:, 1], minlength=n_rel).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        left_mean = (freq / left_cnt).astype(np.float32)
        right_mean = (freq / right_cnt).astype(np.float32)
    return dict(train_list=train_list, head=head, tail=tail, rel=rel, lef_head=lef_head, rig_head=rig_head,
                lef_tail=lef_tail, rig_tail=rig_tail, lef_rel=lef_rel, rig_rel=rig_rel,
                left_mean=left_mean, right_mean=right_mean, n_ent=n_ent, n_rel=n_rel)


def import_prob(path, n_rel, temperature):
    """importProb (Reader.h:26-49): float32 [n_rel, n_rel - 1]."""
    out = np.zeros((n_rel, n_rel - 1), np.float32)
    if lib().orc_import_prob(str(path).encode(), int(n_rel), ctypes.c_float(temperature), _ptr(out)) != 0:
        raise FileNotFoundError(path)
    return out


def sampling(ix, seeds, batch_size, neg_rate=1, neg_rel_rate=0, mode=0, bern=False, train_total=None, prob=None):
    """Base.cpp:161-197. seeds: uint64 per work thread (advanced in place). prob: import_prob's
    table for sampling(..., p=True) (Corrupt.h:111-147), None for p=False."""
    B = batch_size
    n = B * (1 + neg_rate + neg_rel_rate)
    bh = np.zeros(n, np.int64)
    bt = np.zeros(n, np.int64)
    br = np.zeros(n, np.int64)
    by = np.zeros(n, np.float32)
    tl = _i64(ix["train_list"])
    lib().orc_sampling(_ptr(tl), int(train_total if train_total is not None else tl.shape[0]),
                       _ptr(_i64(ix["head"])), _ptr(_i64(ix["tail"])), _ptr(_i64(ix["rel"])),
                       _ptr(ix["lef_head"]), _ptr(ix["rig_head"]), _ptr(ix["lef_tail"]), _ptr(ix["rig_tail"]),
                       _ptr(ix["lef_rel"]), _ptr(ix["rig_rel"]),
                       _ptr(ix["left_mean"]) if bern else None, _ptr(ix["right_mean"]) if bern else None,
                       ix["n_ent"], ix["n_rel"], seeds.ctypes.data_as(ctypes.c_void_p), seeds.shape[0],
                       _ptr(bh), _ptr(bt), _ptr(br), _ptr(by), B, neg_rate, neg_rel_rate, mode,
                       None if prob is None else _ptr(np.ascontiguousarray(prob, np.float32)))
    return bh, bt, br, by


# ------------------------------------------------------ candidate rankings --
def candidate_rank_transe(ent, rel, qh, qr, cand_off, cand_ids):
    ent, rel = _f32(ent), _f32(rel)
    qh, qr, cand_off, cand_ids = _i64(qh), _i64(qr), _i64(cand_off), _i64(cand_ids)
    scores = np.zeros(cand_ids.shape[0], np.float32)
    ranks = np.zeros(qh.shape[0], np.int64)
    lib().orc_candidate_rank_transe(_ptr(ent), _ptr(rel), rel.shape[1], _ptr(qh), _ptr(qr), _ptr(cand_off),
                                    _ptr(cand_ids), qh.shape[0], _ptr(scores), _ptr(ranks))
    return scores, ranks


def cosine_rank(cand_vecs, cand_off, rel_vecs, rel_of_query):
    """ZSLmodule.eval ranking (zsl_module.py:699-706): mean cosine similarity of each
    candidate against the relation's generated vectors; rank = 1 + #(score > true score).
    Float64 restatement (sklearn normalises rows, then X @ Y.T)."""
    X = np.asarray(cand_vecs, np.float64)
    Xn = X / np.maximum(np.linalg.norm(X, axis=1, keepdims=True), 1e-300)
    ranks = np.zeros(len(cand_off) - 1, np.int64)
    scores = np.zeros(X.shape[0], np.float64)
    for q in range(len(cand_off) - 1):
        Y = np.asarray(rel_vecs[rel_of_query[q]], np.float64)
        Yn = Y / np.maximum(np.linalg.norm(Y, axis=1, keepdims=True), 1e-300)
        a, b = cand_off[q], cand_off[q + 1]
        s = (Xn[a:b] @ Yn.T).mean(1)
        scores[a:b] = s
        ranks[q] = 1 + int(np.sum(s[1:] > s[0]))
    return scores, ranks


# ---------------------------------------------------------------- generator --
def _sn_weight(w, u, v, train, eps=1e-12):
    w = np.asarray(w, np.float64)
    u = np.asarray(u, np.float64).copy()
    v = np.asarray(v, np.float64).copy()
    if train:
        v = w.T @ u
        v = v / max(np.linalg.norm(v), eps)
        u = w @ v
        u = u / max(np.linalg.norm(u), eps)
    sigma = u @ (w @ v)
    return w / sigma, u, v


def generator_forward(noise, cls, layers, ln_a, ln_b, train=False, eps=1e-3):
    """UnifiedModel.generate MLP part (module/model.py:679-686) in float64.
    layers: list of (W_orig, bias, u, v) for generate_fc_layer, des_rel_map_layer1, des_rel_map_layer2.
    Returns (out, [(u, v) updated per layer])."""
    x = np.concatenate([np.asarray(noise, np.float64), np.asarray(cls, np.float64)], axis=1)
    uv = []
    for (w, b, u, v) in layers:
        wn, u2, v2 = _sn_weight(w, u, v, train)
        uv.append((u2, v2))
        x = x @ wn.T + np.asarray(b, np.float64)
    if x.shape[1] == 1:
        return x, uv
    mu = x.mean(-1, keepdims=True)
    sd = x.std(-1, ddof=1, keepdims=True)
    out = (x - mu) / (sd + eps) * np.asarray(ln_a, np.float64) + np.asarray(ln_b, np.float64)
    return out, uv


# ----------------------------------------------------------- margin loss ----
def margin_loss(p, n, margin, adv_temperature=None):
    """MarginLoss (module/loss.py:5-28, OpenKE MarginLoss.py:8-33) in float64."""
    p = np.asarray(p, np.float64)
    n = np.asarray(n, np.float64)
    x = np.maximum(p - n, -margin)
    if adv_temperature is None:
        return x.mean() + margin
    w = np.exp(-n * adv_temperature - np.max(-n * adv_temperature, -1, keepdims=True))
    w = w / w.sum(-1, keepdims=True)
    return (w * x).sum(-1).mean() + margin
