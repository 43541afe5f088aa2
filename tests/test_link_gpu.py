"""GPU parity of the link-prediction sweep (libmmre_hip.so, through the C ABI) against the
oracle (oracle/) and the reference's golden vectors (tests/golden/link_small.npz).

Bar: predicted scores bit-identical to the oracle's canonical arithmetic; raw / filtered /
type-constrained counts exact; Test.h metrics bit-identical to the reference Base.so's on the
golden dataset; reference torch scores within 1e-4 (relative above 1).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

GOLD_CFG = {
    "transe": dict(model="transe", norm=True, margin=None),
    "transe_nonorm_margin": dict(model="transe", norm=False, margin=5.0),
    "transe_l2": dict(model="transe_l2", norm=True, margin=None),
    "distmult": dict(model="distmult", norm=False, margin=None),
    "complex": dict(model="complex", norm=False, margin=None),
    "rotate": dict(model="rotate", norm=False, margin=6.0),
}


def _spec_from(model, ent, rel, ent_im=None, rel_im=None, norm=False, margin=None, dim=None, eps=2.0):
    from mmre.link import ScoreSpec, rotate_phase_denom
    import oracle
    dev = torch.device("cuda:0")
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
    d = dim if dim is not None else rel.shape[1]
    pk = oracle.pred_kind(model, margin is not None)
    pd = rotate_phase_denom(margin, eps, d) if model == "rotate" else 0.0
    return ScoreSpec(model=model, ent=t(ent), rel=t(rel), dim=d, ent_im=t(ent_im), rel_im=t(rel_im), norm_flag=norm,
                     pred_kind=pk, margin=float(margin or 0.0), phase_denom=pd)


def _tables(g, name):
    if name == "complex":
        return (g[f"{name}.ent_re_embeddings.weight"], g[f"{name}.rel_re_embeddings.weight"],
                g[f"{name}.ent_im_embeddings.weight"], g[f"{name}.rel_im_embeddings.weight"])
    return g[f"{name}.ent_embeddings.weight"], g[f"{name}.rel_embeddings.weight"], None, None


def _run(spec, qh, qr, qt, qm, index=None, tc=False, scores=True, grouped=True, q_rows=True):
    from mmre.link import LinkSweep
    dev = spec.ent.device
    filt = masks = None
    if index is not None:
        lists = index.groups(qh, qr, qt, qm) if grouped else index.filters(qh, qr, qt, qm)
        filt = tuple(torch.from_numpy(a).to(dev) for a in lists)
        if tc:
            masks = tuple(torch.from_numpy(m).to(dev) for m in index.type_masks())
    sw = LinkSweep(spec)
    bufs = sw.alloc_queries(len(qh))
    res = sw.run(*(torch.from_numpy(np.asarray(x, np.int64)).to(dev) for x in (qh, qr, qt)),
                 torch.from_numpy(np.asarray(qm, np.int8)).to(dev), filt=filt, type_masks=masks,
                 return_scores=scores, q_rows=q_rows, buffers=bufs)
    torch.cuda.synchronize()
    out = {k: (v.cpu().numpy() if v is not None else None) for k, v in res.items()}
    st = sw.l1q_stats(bufs)
    if st is not None:  # the rescoring's range guard never fires
        assert st["guarded"] == 0, st
    out["l1q"] = st
    return out


@pytest.mark.parametrize("name", list(GOLD_CFG))
@pytest.mark.parametrize("tc", [0, 1])
@pytest.mark.parametrize("grouped", [0, 1])
def test_golden_link_small(golden, oracle_mod, name, tc, grouped):
    from mmre.data import OpenKEDataset
    from mmre.link import FilterIndex, link_metrics
    g = golden("link_small")
    c = GOLD_CFG[name]
    ent, rel, ent_im, rel_im = _tables(g, name)
    dim = 16 if name == "rotate" else rel.shape[1]
    spec = _spec_from(c["model"], ent, rel, ent_im, rel_im, norm=c["norm"], margin=c["margin"], dim=dim)
    ds = OpenKEDataset(os.path.join(GOLDEN, "data", "small"))
    index = FilterIndex(*ds.all_triples(), ds.n_ent, ds.n_rel, ds.type_heads, ds.type_tails)
    qh, qr, qt = g["qh"], g["qr"], g["qt"]
    n = len(qh)
    QH, QR, QT = (np.concatenate([x, x]) for x in (qh, qr, qt))
    QM = np.concatenate([np.zeros(n, np.int8), np.ones(n, np.int8)])
    out = _run(spec, QH, QR, QT, QM, index=index, tc=bool(tc), grouped=bool(grouped), q_rows=bool(grouped))
    okw = dict(ent_im=ent_im, rel_im=rel_im, norm_flag=c["norm"], margin=c["margin"])
    if c["model"] == "rotate":
        okw["phase_denom"] = spec.phase_denom
    trip = np.concatenate([ds.train, ds.valid, ds.test])
    hrt = oracle_mod.sorted_hrt(trip[:, 0], trip[:, 2], trip[:, 1])
    counts = {}
    for side, mode, sl in (("head", "head_batch", slice(0, n)), ("tail", "tail_batch", slice(n, 2 * n))):
        o_pred = oracle_mod.link_predict(c["model"], mode, ent, rel, qh, qr, qt, **okw)
        # 1. scores: bit-identical to the oracle (canonical arithmetic), within 1e-4 of the reference
        assert np.array_equal(out["scores"][sl], o_pred), np.abs(out["scores"][sl] - o_pred).max()
        ref = g[f"{name}_pred_{side}"]
        assert np.all(np.abs(out["scores"][sl] - ref) <= 1e-4 * np.maximum(1, np.abs(ref)))
        # 2. counts: exact vs the oracle's Test.h restatement
        toff = tids = None
        if tc:
            lists = ds.type_heads if side == "head" else ds.type_tails
            toff = np.cumsum([0] + [len(x) for x in lists])
            tids = np.concatenate([np.asarray(x, np.int64) for x in lists])
        o_c = oracle_mod.test_rank(mode, o_pred, qh, qr, qt, hrt, toff, tids)
        got = out["counts"][:, sl].T
        cols = [0, 1, 2, 3] if tc else [0, 1]
        assert np.array_equal(got[:, cols], o_c[:, cols])
        counts[side] = out["counts"][:, sl]
    # 3. metrics: Test.h float semantics; equal to the reference Base.so where no near-tie
    m = link_metrics(counts["head"], counts["tail"])
    grp = m["filter_tc" if tc else "filter"]
    got = np.array([grp[k] for k in ("mrr", "mr", "hit10", "hit3", "hit1")], np.float32)
    ref_counts_equal = (np.array_equal(counts["head"][[0, 1]].T, g[f"{name}_tc{tc}_head_counts"][:, :2]) and
                        np.array_equal(counts["tail"][[0, 1]].T, g[f"{name}_tc{tc}_tail_counts"][:, :2]))
    if ref_counts_equal:
        assert np.array_equal(got, g[f"{name}_tc{tc}_metrics"])
    # hit@{1,3,10} are count thresholds: they must match the reference exactly
    assert np.array_equal(got[2:], g[f"{name}_tc{tc}_metrics"][2:])


def _random_case(model, E, R, d, Q, seed, norm=False, margin=None, with_ties=False):
    rng = np.random.default_rng(seed)
    ent_w = 2 * d if model == "rotate" else d
    ent = rng.uniform(-0.5, 0.5, (E, ent_w)).astype(np.float32)
    rel = rng.uniform(-0.5, 0.5, (R, d)).astype(np.float32)
    ent_im = rng.uniform(-0.5, 0.5, (E, d)).astype(np.float32) if model == "complex" else None
    rel_im = rng.uniform(-0.5, 0.5, (R, d)).astype(np.float32) if model == "complex" else None
    qh = rng.integers(0, E, Q)
    qr = rng.integers(0, R, Q)
    qt = rng.integers(0, E, Q)
    qm = rng.integers(0, 2, Q).astype(np.int8)
    if with_ties:  # duplicate rows: exact ties with the truth must not count (strict <)
        for i in range(0, Q, 7):
            tgt = qh[i] if qm[i] == 0 else qt[i]
            dup = (tgt + 1 + i) % E
            ent[dup] = ent[tgt]
            if ent_im is not None:
                ent_im[dup] = ent_im[tgt]
    return ent, rel, ent_im, rel_im, qh, qr, qt, qm


@pytest.mark.parametrize("model,E,d,Q,norm,margin", [
    ("transe", 1000, 200, 300, True, None),
    ("transe", 333, 100, 129, False, 4.0),
    ("transe", 129, 7, 1, True, None),
    ("transe_l2", 700, 64, 257, True, None),
    ("distmult", 1000, 200, 300, False, None),
    ("distmult", 250, 13, 77, False, None),
    ("complex", 900, 200, 200, False, None),
    ("rotate", 600, 64, 150, False, 6.0),
])
def test_random_bit_exact(oracle_mod, model, E, d, Q, norm, margin):
    from mmre.link import FilterIndex
    ent, rel, ent_im, rel_im, qh, qr, qt, qm = _random_case(model, E, 11, d, Q, seed=E + d + Q, norm=norm,
                                                            margin=margin, with_ties=True)
    spec = _spec_from(model, ent, rel, ent_im, rel_im, norm=norm, margin=margin, dim=d)
    rng = np.random.default_rng(5)
    th, tr, tt = rng.integers(0, E, 4 * E), rng.integers(0, 11, 4 * E), rng.integers(0, E, 4 * E)
    th = np.concatenate([th, qh]); tr = np.concatenate([tr, qr]); tt = np.concatenate([tt, qt])
    index = FilterIndex(th, tr, tt, E, 11)
    out = _run(spec, qh, qr, qt, qm, index=index)
    hrt = oracle_mod.sorted_hrt(th, tr, tt)
    okw = dict(ent_im=ent_im, rel_im=rel_im, norm_flag=norm, margin=margin,
               phase_denom=spec.phase_denom)
    for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
        sel = qm == mode_id
        if not sel.any():
            continue
        o_pred = oracle_mod.link_predict(model, mode, ent, rel, qh[sel], qr[sel], qt[sel], **okw)
        assert np.array_equal(out["scores"][sel], o_pred)
        o_c = oracle_mod.test_rank(mode, o_pred, qh[sel], qr[sel], qt[sel], hrt)
        assert np.array_equal(out["counts"][:, sel].T[:, :2], o_c[:, :2])
        tv = out["truth"][sel]
        truth_ids = qh[sel] if mode_id == 0 else qt[sel]
        assert np.array_equal(tv, o_pred[np.arange(sel.sum()), truth_ids])


def test_full_size_c2_properties(oracle_mod):
    """BASELINE config C2 at full size (FB15K-237-ZS, E=14,208, d=200, Q=35,192 sweeps):
    size-independent properties on every query + oracle parity on a seeded subset."""
    from mmre.data import load_zs_test
    from mmre.link import FilterIndex
    z = load_zs_test("FB15K-237-ZS")
    E, R = int(z["n_ent"]), int(z["n_rel"])
    rng = np.random.default_rng(0)
    bound = np.sqrt(6.0 / (E + 200))
    ent = rng.uniform(-bound, bound, (E, 200)).astype(np.float32)
    rel = rng.uniform(-np.sqrt(6.0 / (R + 200)), np.sqrt(6.0 / (R + 200)), (R, 200)).astype(np.float32)
    h, r, t = z["h"].astype(np.int64), z["r"].astype(np.int64), z["t"].astype(np.int64)
    n = len(h)
    qh, qr, qt = np.concatenate([h, h]), np.concatenate([r, r]), np.concatenate([t, t])
    qm = np.concatenate([np.zeros(n, np.int8), np.ones(n, np.int8)])
    index = FilterIndex(h, r, t, E, R)
    spec = _spec_from("transe", ent, rel, norm=True, dim=200)
    out = _run(spec, qh, qr, qt, qm, index=index, scores=False)
    c = out["counts"]
    assert np.all(c[0] >= c[1]) and np.all(c[1] >= 0) and np.all(c[0] <= E - 1)
    off, ids = index.filters(qh, qr, qt, qm)
    assert np.all(c[0] - c[1] <= np.diff(off))
    sub = rng.choice(2 * n, 48, replace=False)
    hrt = oracle_mod.sorted_hrt(h, r, t)
    for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
        s = sub[qm[sub] == mode_id]
        o_pred = oracle_mod.link_predict("transe", mode, ent, rel, qh[s], qr[s], qt[s], norm_flag=True)
        o_c = oracle_mod.test_rank(mode, o_pred, qh[s], qr[s], qt[s], hrt)
        assert np.array_equal(c[:, s].T[:, :2], o_c[:, :2])


def test_rotate_zero_and_tiny_magnitudes(oracle_mod):
    """RotatE's fast magnitude is exact only for inputs >= 2^-96; tiles that see 0, tiny or
    overflowing inputs are recomputed with sqrtf. Relation 0 has phase 0 (an exact identity
    rotation), so a query's anchor scores v = 0 on every k, and near-copies of the anchor
    score v ~ 1e-44 (subnormal) and ~1e-31 (below 2^-96): scores must stay bit-identical."""
    rng = np.random.default_rng(11)
    E, R, d, margin = 300, 5, 32, 6.0
    er = (margin + 2.0) / (2 * d)
    ent = rng.uniform(-er, er, (E, 2 * d)).astype(np.float32)
    rel = rng.uniform(-(margin + 2.0) / d, (margin + 2.0) / d, (R, d)).astype(np.float32)
    rel[0] = 0.0
    ent[5] = ent[3]
    ent[5, ::3] += np.float32(1e-22)       # dr ~ 1e-22 -> v ~ 1e-44 (subnormal)
    ent[6] = ent[3]
    ent[6, 1::4] += np.float32(3e-16)      # v ~ 1e-31 < 2^-96
    ent[7] = ent[4]
    qh = np.array([3, 3, 4, 10, 3, 4], np.int64)
    qr = np.array([0, 0, 0, 1, 2, 0], np.int64)
    qt = np.array([4, 3, 3, 12, 5, 4], np.int64)
    qm = np.array([1, 0, 1, 0, 1, 0], np.int8)
    spec = _spec_from("rotate", ent, rel, margin=margin, dim=d)
    out = _run(spec, qh, qr, qt, qm)
    for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
        sel = qm == mode_id
        o_pred = oracle_mod.link_predict("rotate", mode, ent, rel, qh[sel], qr[sel], qt[sel], margin=margin,
                                         phase_denom=spec.phase_denom)
        assert np.array_equal(out["scores"][sel].view(np.uint32), o_pred.view(np.uint32))


@pytest.mark.parametrize("model", ["transe", "distmult"])
def test_tiny_tables_and_empty_query_set(oracle_mod, model):
    """Edge sizes: a single-entity table (every sweep's only candidate is its truth: rank 0),
    two entities, and an empty query set (a rank owning no test relation) that launches nothing."""
    from mmre.link import FilterIndex
    rng = np.random.default_rng(3)
    for E in (1, 2):
        ent = rng.uniform(-0.5, 0.5, (E, 8)).astype(np.float32)
        rel = rng.uniform(-0.5, 0.5, (2, 8)).astype(np.float32)
        qh = np.zeros(4, np.int64) if E == 1 else np.array([0, 1, 0, 1])
        qr = np.array([0, 1, 0, 1], np.int64)
        qt = np.zeros(4, np.int64) if E == 1 else np.array([1, 0, 1, 0])
        qm = np.array([0, 0, 1, 1], np.int8)
        spec = _spec_from(model, ent, rel, norm=model == "transe")
        index = FilterIndex(qh, qr, qt, E, 2)
        out = _run(spec, qh, qr, qt, qm, index=index)
        hrt = oracle_mod.sorted_hrt(qh, qr, qt)
        for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
            sel = qm == mode_id
            o = oracle_mod.link_predict(model, mode, ent, rel, qh[sel], qr[sel], qt[sel], norm_flag=model == "transe")
            assert np.array_equal(out["scores"][sel], o)
            oc = oracle_mod.test_rank(mode, o, qh[sel], qr[sel], qt[sel], hrt)
            assert np.array_equal(out["counts"][:, sel].T[:, :2], oc[:, :2])
        if E == 1:
            assert (out["counts"] == 0).all()
    e = np.zeros(0, np.int64)
    out = _run(spec, e, e, e, np.zeros(0, np.int8), index=index)
    assert out["counts"].shape == (4, 0) and out["scores"].shape == (0, 2)


def test_pipelined_launch_finish_matches_run():
    """ShardedLinkEvaluation.launch/finish (two evaluations in flight, alternating pinned
    buffers, as bench.py drives it) gives the same counts and metrics as run(), for two
    different model snapshots whose tickets overlap."""
    from mmre.data import OpenKEDataset
    from mmre.link import FilterIndex
    from mmre.sharding import ShardedLinkEvaluation
    ds = OpenKEDataset(os.path.join(GOLDEN, "data", "small"))
    h, r, t = ds.test_list()
    index = FilterIndex(*ds.all_triples(), ds.n_ent, ds.n_rel)
    rng = np.random.default_rng(3)
    evs = []
    for _ in range(2):
        ent = rng.uniform(-0.3, 0.3, (ds.n_ent, 64)).astype(np.float32)
        rel = rng.uniform(-0.3, 0.3, (ds.n_rel, 64)).astype(np.float32)
        evs.append(ShardedLinkEvaluation(_spec_from("transe", ent, rel, norm=True, dim=64), h, r, t, index=index,
                                         device="cuda:0"))
    ref = [e.run() for e in evs]
    ev = evs[0]
    a = ev.launch()
    b = ev.launch()
    with pytest.raises(RuntimeError):
        ev.launch()  # a third ticket would overwrite a pinned buffer still unread
    ma, ca = ev.finish(a)
    mb, cb = ev.finish(b)
    with pytest.raises(RuntimeError):
        ev.finish(b)  # a ticket is finished once
    assert np.array_equal(ca, ref[0][1]) and np.array_equal(cb, ref[0][1])
    assert ma == ref[0][0] and mb == ref[0][0]
    # overlapping tickets of two snapshots keep their own buffers
    ta, tb = evs[0].launch(), evs[1].launch()
    (m0, c0), (m1, c1) = evs[0].finish(ta), evs[1].finish(tb)
    assert np.array_equal(c0, ref[0][1]) and np.array_equal(c1, ref[1][1]) and m1 == ref[1][0]


@pytest.mark.parametrize("config", ["c3", "c4", "c5"])
def test_full_size_configs(oracle_mod, config):
    """BASELINE configs C3 (DB15K-ZS ComplEx d=200, MFMA), C4 (FB15K-237-ZS RotatE d=512) and C5
    (synthetic |E| = 1M DistMult d=256, MFMA) at full size, through the bench's workloads:
    size-independent properties on every sweep (filtered <= raw <= E - 1, raw - filtered <= the
    query's filter list) + bit-exact counts and truth scores vs the oracle on a seeded subset."""
    from mmre.link import FilterIndex
    from mmre.workloads import synthetic_large, zs_workload
    if config == "c5":
        w = synthetic_large(generator_device="cuda:0")  # relation rows from the HIP generator
    else:
        w = zs_workload(*{"c3": ("DB15K-ZS", "complex", 200), "c4": ("FB15K-237-ZS", "rotate", 512)}[config])
    model, E, R = w["model"], int(w["n_ent"]), int(w["n_rel"])
    np_ = lambda k: None if k not in w else w[k].numpy()
    ent, rel, ent_im, rel_im = np_("ent"), np_("rel"), np_("ent_im"), np_("rel_im")
    margin = w.get("margin")
    spec = _spec_from(model, ent, rel, ent_im, rel_im, margin=margin, dim=w["dim"], eps=w.get("epsilon", 2.0))
    h, r, t = (np.asarray(w[k], np.int64) for k in ("test_h", "test_r", "test_t"))
    n = len(h)
    qh, qr, qt = np.concatenate([h, h]), np.concatenate([r, r]), np.concatenate([t, t])
    qm = np.concatenate([np.zeros(n, np.int8), np.ones(n, np.int8)])
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], E, R)
    out = _run(spec, qh, qr, qt, qm, index=index, scores=False)
    c = out["counts"]
    assert np.all(c[0] >= c[1]) and np.all(c[1] >= 0) and np.all(c[0] <= E - 1)
    off, _ = index.filters(qh, qr, qt, qm)
    assert np.all(c[0] - c[1] <= np.diff(off))
    rng = np.random.default_rng(1)
    sub = rng.choice(2 * n, 8 if config == "c5" else 24, replace=False)
    hrt = oracle_mod.sorted_hrt(w["filter_h"], w["filter_r"], w["filter_t"])
    okw = dict(ent_im=ent_im, rel_im=rel_im, norm_flag=False, margin=margin, phase_denom=spec.phase_denom)
    for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
        s = np.sort(sub[qm[sub] == mode_id])
        if len(s) == 0:
            continue
        o_pred = oracle_mod.link_predict(model, mode, ent, rel, qh[s], qr[s], qt[s], **okw)
        o_c = oracle_mod.test_rank(mode, o_pred, qh[s], qr[s], qt[s], hrt)
        assert np.array_equal(c[:, s].T[:, :2], o_c[:, :2])
        truth_ids = qh[s] if mode_id == 0 else qt[s]
        assert np.array_equal(out["truth"][s], o_pred[np.arange(len(s)), truth_ids])


def test_c1_config_full_oracle(oracle_mod):
    """BASELINE configs[0] (C1): FB15K-237-ZS TransE d=100 on the first 1,000 test triples in
    Test.h order (the reference's OpenKE Tester path, Tester.py:70-91), tables trained by this
    build's trainer so ranks are not degenerate, evaluated as bench.py --config c1 does
    (ShardedLinkEvaluation: filter groups, pipelined launch/finish): every one of the 2,000
    sweeps' raw / filtered counts equal the oracle's, and so the Test.h metrics."""
    from mmre.link import FilterIndex, link_metrics
    from mmre.sharding import ShardedLinkEvaluation
    from mmre.workloads import train_transe, zs_workload
    w = zs_workload("FB15K-237-ZS", "transe", 100, n_test=1000)
    w["norm_flag"] = True
    train_transe(w, "cuda:0", steps=100)
    E, R, n = int(w["n_ent"]), int(w["n_rel"]), len(w["test_h"])
    assert n == 1000
    ent, rel = w["ent"].numpy(), w["rel"].numpy()
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], E, R)
    ev = ShardedLinkEvaluation(_spec_from("transe", ent, rel, norm=True, dim=100), w["test_h"], w["test_r"],
                               w["test_t"], index=index, device="cuda:0")
    metrics, counts = ev.finish(ev.launch())
    h, r, t = (np.asarray(w[k], np.int64) for k in ("test_h", "test_r", "test_t"))
    hrt = oracle_mod.sorted_hrt(np.asarray(w["filter_h"], np.int64), np.asarray(w["filter_r"], np.int64),
                                np.asarray(w["filter_t"], np.int64))
    oc = []
    for mode in ("head_batch", "tail_batch"):
        o_pred = oracle_mod.link_predict("transe", mode, ent, rel, h, r, t, norm_flag=True)
        oc.append(oracle_mod.test_rank(mode, o_pred, h, r, t, hrt)[:, :2].T)
    o_counts = np.concatenate(oc, 1)
    assert np.array_equal(counts[:2], o_counts)
    z = np.zeros((2, n), np.int32)
    o_metrics = link_metrics(np.concatenate([o_counts[:, :n], z]).astype(np.int32),
                             np.concatenate([o_counts[:, n:], z]).astype(np.int32))
    assert metrics["filter"] == o_metrics["filter"] and metrics["raw"] == o_metrics["raw"]
    assert metrics["filter"]["hit10"] > 0.5      # trained tables: truths rank near the top
