"""GPU parity of the sweep's filters (csrc/link.hip): the count-only RotatE sweeps sum the raw
v_sqrt_f32 -- within 1 ulp of sqrtf (scripts/probes/sqrt_ulp.hip, exhaustive) -- and the
count-only TransE L1 sweeps sum |code differences| of 8-bit (v_sad_u8) or 16-bit (v_sad_u16)
quantized planes (mmre_link_sweep_l1q; the width picked on the device by a sampled probe, or
forced with MMRE_L1_BITS); both rescore with the canonical chain every pair whose prediction the
error bound cannot place on one side of the threshold.

Bar: raw / filtered / type-constrained counts bit-equal to the score-storing (exact) sweep's
and to the oracle's Test.h restatement, on tables built to put many pairs inside the bound:
exact copies of the truth row (exact ties: strict < must not count them), copies one ulp away
in a few coordinates (scores a few ulps from the threshold), zero rows, rows of subnormal and
of overflowing magnitude, NaN rows, and an identity rotation (v = 0 on every k).
"""
import os

import numpy as np
import pytest

from test_link_gpu import _run, _spec_from

pytestmark = pytest.mark.gpu


def _adversarial(E=1500, R=6, d=48, Q=257, seed=0, margin=6.0, model="rotate", huge=True):
    rng = np.random.default_rng(seed)
    er = (margin + 2.0) / (2 * d)
    ent = rng.uniform(-er, er, (E, 2 * d if model == "rotate" else d)).astype(np.float32)
    rel = rng.uniform(-(margin + 2.0) / d, (margin + 2.0) / d, (R, d)).astype(np.float32)
    rel[0] = 0.0                                       # RotatE phase 0 / TransE r = 0: v = 0 at the anchor
    qh, qr, qt = rng.integers(0, E, Q), rng.integers(0, R, Q), rng.integers(0, E, Q)
    qm = rng.integers(0, 2, Q).astype(np.int8)
    free = iter(rng.permutation(np.arange(E)))
    used = set(qh.tolist()) | set(qt.tolist())
    nxt = lambda: next(e for e in free if e not in used)
    for i in range(0, Q, 3):
        truth = qh[i] if qm[i] == 0 else qt[i]
        for _ in range(3):                             # exact ties with the truth
            ent[nxt()] = ent[truth]
        for k in range(4):                             # a few ulps away from the truth's score
            e = nxt()
            ent[e] = ent[truth]
            cols = rng.choice(ent.shape[1], 1 + k, replace=False)
            bump = np.where(rng.random(len(cols)) < 0.5, -np.inf, np.inf).astype(np.float32)
            ent[e, cols] = np.nextafter(ent[e, cols], bump)
    for _ in range(5):
        ent[nxt()] = 0.0
    e = nxt(); ent[e] = ent[qt[0]]; ent[e, ::5] += np.float32(1e-22)     # v subnormal
    e = nxt(); ent[e] = ent[qt[1]]; ent[e, 1::4] += np.float32(3e-16)    # v < 2^-96
    if huge:
        e = nxt(); ent[e] = 3e19                                          # v = inf
        e = nxt(); ent[e, 7] = np.nan
    return ent, rel, qh, qr, qt, qm


@pytest.mark.parametrize("model,seed,huge", [("rotate", 0, True), ("rotate", 1, True), ("transe", 0, False),
                                             ("transe", 1, False), ("transe", 2, True)])
def test_fast_filter_counts_equal_exact_sweep_and_oracle(oracle_mod, monkeypatch, model, seed, huge):
    """huge: a row of 3e19 and a NaN -- for TransE these make the quantization scale
    non-finite, so every pair is rescored (slow, exact). TransE runs every code width: 8-bit,
    16-bit and the probe's choice."""
    for bits in (("8", "16", None) if model == "transe" else (None,)):
        if bits is None:
            monkeypatch.delenv("MMRE_L1_BITS", raising=False)
        else:
            monkeypatch.setenv("MMRE_L1_BITS", bits)
        _fast_filter_case(oracle_mod, model, seed, huge)


def _fast_filter_case(oracle_mod, model, seed, huge):
    from mmre.link import FilterIndex
    margin = 6.0 if model == "rotate" else None
    ent, rel, qh, qr, qt, qm = _adversarial(seed=seed, margin=margin or 6.0, model=model, huge=huge)
    E, R, d = ent.shape[0], rel.shape[0], rel.shape[1]
    rng = np.random.default_rng(seed + 10)
    fh, fr, ft = rng.integers(0, E, 3 * E), rng.integers(0, R, 3 * E), rng.integers(0, E, 3 * E)
    fh, fr, ft = np.concatenate([fh, qh]), np.concatenate([fr, qr]), np.concatenate([ft, qt])
    heads = [np.unique(np.concatenate([rng.choice(E, E // 3, replace=False), qh[qr == r]])) for r in range(R)]
    tails = [np.unique(np.concatenate([rng.choice(E, E // 3, replace=False), qt[qr == r]])) for r in range(R)]
    index = FilterIndex(fh, fr, ft, E, R, heads, tails)
    spec = _spec_from(model, ent, rel, margin=margin, dim=d, norm=model == "transe")
    exact = _run(spec, qh, qr, qt, qm, index=index, tc=True, scores=True)
    fast = _run(spec, qh, qr, qt, qm, index=index, tc=True, scores=False)
    plain = _run(spec, qh, qr, qt, qm, index=index, tc=False, scores=False)
    assert np.array_equal(fast["counts"], exact["counts"])
    assert np.array_equal(plain["counts"][:2], exact["counts"][:2])
    assert np.array_equal(fast["truth"].view(np.uint32), exact["truth"].view(np.uint32))
    hrt = oracle_mod.sorted_hrt(fh, fr, ft)
    for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
        sel = qm == mode_id
        o_pred = oracle_mod.link_predict(model, mode, ent, rel, qh[sel], qr[sel], qt[sel], margin=margin,
                                         phase_denom=spec.phase_denom, norm_flag=model == "transe")
        lists = heads if mode_id == 0 else tails
        toff = np.cumsum([0] + [len(x) for x in lists])
        tids = np.concatenate([np.asarray(x, np.int64) for x in lists])
        o_c = oracle_mod.test_rank(mode, o_pred, qh[sel], qr[sel], qt[sel], hrt, toff, tids)
        assert np.array_equal(fast["counts"][:, sel].T, o_c)
    # the construction really exercises the rescoring: many truths have exact ties
    assert (exact["counts"][0] < E - 1).all()


def test_l1_filter_on_and_off_and_entity_slices(oracle_mod, monkeypatch):
    """TransE L1: the integer-filter sweep equals the f32 sweep (MMRE_L1_FILTER=0) on the whole
    table and on entity slices (mmre_link_sweep_l1q with e_begin / e_end), whose counts sum to
    the whole-table ones; the margin prediction kind takes the generic epilogue. Every code
    width (MMRE_L1_BITS 8, 16, the probe's choice)."""
    import torch
    from mmre.link import FilterIndex, LinkSweep
    for margin, bits in ((None, "8"), (None, "16"), (None, None), (4.0, "8"), (4.0, "16"), (4.0, None)):
        if bits is None:
            monkeypatch.delenv("MMRE_L1_BITS", raising=False)
        else:
            monkeypatch.setenv("MMRE_L1_BITS", bits)
        ent, rel, qh, qr, qt, qm = _adversarial(E=2100, d=40, Q=200, seed=5, model="transe", huge=False)
        E, R = ent.shape[0], rel.shape[0]
        index = FilterIndex(qh, qr, qt, E, R)
        spec = _spec_from("transe", ent, rel, margin=margin, dim=40, norm=True)
        on = _run(spec, qh, qr, qt, qm, index=index, scores=False)
        monkeypatch.setenv("MMRE_L1_FILTER", "0")
        off = _run(spec, qh, qr, qt, qm, index=index, scores=False)
        monkeypatch.delenv("MMRE_L1_FILTER")
        assert np.array_equal(on["counts"], off["counts"])
        dev = spec.ent.device
        tq = lambda a, dt=np.int64: torch.from_numpy(np.asarray(a, dt)).to(dev)
        total = np.zeros_like(on["counts"])
        for e0, e1 in ((0, 512), (512, 1536), (1536, E)):
            filt = tuple(torch.from_numpy(a).to(dev) for a in index.groups(qh, qr, qt, qm, entity_range=(e0, e1)))
            sw = LinkSweep(spec)
            res = sw.run(tq(qh), tq(qr), tq(qt), tq(qm, np.int8), filt=filt, entity_range=(e0, e1))
            total += res["counts"].cpu().numpy()
        assert np.array_equal(total, on["counts"])


def _c2_eval(w, dev, norm_flag):
    from mmre.link import FilterIndex, HEAD, TAIL, LinkSweep, ScoreSpec
    import torch
    n = len(w["test_h"])
    to = lambda a, dt=np.int64: torch.from_numpy(np.asarray(a, dt)).to(dev)
    qh, qr, qt = (np.r_[w[k], w[k]] for k in ("test_h", "test_r", "test_t"))
    qm = np.r_[np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)]
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
    filt = tuple(to(a, a.dtype) for a in index.groups(qh, qr, qt, qm))
    spec = ScoreSpec(model="transe", ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=int(w["dim"]),
                     norm_flag=norm_flag, pred_kind=0)
    sw = LinkSweep(spec)
    bufs = sw.alloc_queries(2 * n)
    args = (to(qh), to(qr), to(qt), to(qm, np.int8))

    def run(reps=5):
        ts = []
        for _ in range(reps):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            sw.run(*args, filt=filt, buffers=bufs, sweep_events=ev)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        st = sw.l1q_stats(bufs)
        assert st is None or st["guarded"] == 0, st
        return bufs["counts"].cpu().numpy().copy(), float(np.median(ts)), st
    return sw, run


def test_l1_filter_outlier_row_falls_back_to_f32(monkeypatch):
    """the 16-bit codes span M = max |x| of both planes, so ONE outlier row
    (a drifted norm_flag=False table) would stretch the code step for every pair and leave most
    of them to the one-at-a-time rescoring. The quantization pass detects it (M > 128 x mean|x|)
    on the device and the sweep runs the f32 path instead: counts unchanged, time within 1.1x of
    the f32 sweep (MMRE_L1_FILTER=0). The ordinary table keeps the filter, with its undecided
    pairs counted."""
    import torch
    from mmre.workloads import zs_workload
    dev = torch.device("cuda:0")
    w = zs_workload("FB15K-237-ZS", "transe", 200)
    _, run = _c2_eval(w, dev, norm_flag=False)
    c_plain, t_plain, st_plain = run()
    assert st_plain is not None and not st_plain["fallback"], st_plain
    w["ent"] = w["ent"].clone()
    w["ent"][123] *= 1000.0                               # one drifted entity row
    _, run = _c2_eval(w, dev, norm_flag=False)
    c_out, t_out, st_out = run()
    assert st_out["fallback"] and st_out["undecided"] == 0, st_out
    monkeypatch.setenv("MMRE_L1_FILTER", "0")
    _, run32 = _c2_eval(w, dev, norm_flag=False)
    c_32, t_32, st_32 = run32()
    assert st_32 is None
    assert np.array_equal(c_out, c_32)
    print(f"L1 filter: plain table {t_plain:.3f} ms ({st_plain['undecided']} undecided pairs); outlier table "
          f"{t_out:.3f} ms (fallback) vs f32 sweep {t_32:.3f} ms")
    assert t_out <= 1.1 * t_32


def test_l1_code_width_probe_picks_16_bit_on_untrained_tables(monkeypatch):
    """The 8-bit codes' band (257x the 16-bit one) holds tens of percent of the pairs when the
    truths rank mid-table (xavier-init C2 tables): the probe sees it and the 16-bit codes run,
    counts equal to both forced widths and the f32 sweep, time within 1.15x of the forced 16-bit
    sweep (the probe, the 16-bit quantization and the 8-bit launch's early exit are the extra)."""
    from mmre.workloads import zs_workload
    import torch
    dev = torch.device("cuda:0")
    w = zs_workload("FB15K-237-ZS", "transe", 200)
    res = {}
    for bits in (None, "8", "16"):
        if bits is None:
            monkeypatch.delenv("MMRE_L1_BITS", raising=False)
        else:
            monkeypatch.setenv("MMRE_L1_BITS", bits)
        _, run = _c2_eval(w, dev, norm_flag=True)
        res[bits] = run()
    monkeypatch.delenv("MMRE_L1_BITS", raising=False)
    monkeypatch.setenv("MMRE_L1_FILTER", "0")
    _, run32 = _c2_eval(w, dev, norm_flag=True)
    c32, t32, _ = run32()
    (ca, ta, sa), (c8, t8, s8), (c16, t16, s16) = res[None], res["8"], res["16"]
    print(f"xavier C2: auto {ta:.3f} ms ({sa}), 8-bit {t8:.3f} ms ({s8}), 16-bit {t16:.3f} ms ({s16}), f32 {t32:.3f} ms")
    assert sa["bits"] == 16 and s8["bits"] == 8 and s16["bits"] == 16
    assert np.array_equal(ca, c32) and np.array_equal(c8, c32) and np.array_equal(c16, c32)
    assert ta <= 1.15 * t16


def _adversarial_dot(model, E=2300, R=5, d=48, Q=300, seed=0, nonfinite=True):
    """DistMult / ComplEx tables that put many pairs inside the split-bf16 bound: exact copies of
    the truth row (exact ties), copies a few ulps away, zero rows, rows below the split's 2^-60
    cut, subnormal values, and (nonfinite) a row whose products overflow and a NaN."""
    rng = np.random.default_rng(seed)
    two = model == "complex"
    ent = rng.normal(0, 0.3, (E, d)).astype(np.float32)
    ent_im = rng.normal(0, 0.3, (E, d)).astype(np.float32) if two else None
    rel = rng.normal(0, 0.5, (R, d)).astype(np.float32)
    rel_im = rng.normal(0, 0.5, (R, d)).astype(np.float32) if two else None
    rel[0] = 1.0                                        # DistMult r = 1: scores are plain dot products
    qh, qr, qt = rng.integers(0, E, Q), rng.integers(0, R, Q), rng.integers(0, E, Q)
    qm = rng.integers(0, 2, Q).astype(np.int8)
    free = iter(rng.permutation(np.arange(E)))
    used = set(qh.tolist()) | set(qt.tolist())
    nxt = lambda: next(e for e in free if e not in used)
    tabs = [ent] + ([ent_im] if two else [])
    for i in range(0, Q, 3):
        truth = qh[i] if qm[i] == 0 else qt[i]
        for _ in range(3):                              # exact ties with the truth
            e = nxt()
            for t in tabs:
                t[e] = t[truth]
        for k in range(4):                              # a few ulps away
            e = nxt()
            for t in tabs:
                t[e] = t[truth]
            cols = rng.choice(d, 1 + k, replace=False)
            bump = np.where(rng.random(len(cols)) < 0.5, -np.inf, np.inf).astype(np.float32)
            ent[e, cols] = np.nextafter(ent[e, cols], bump)
    for _ in range(4):
        e = nxt()
        for t in tabs:
            t[e] = 0.0
    e = nxt(); ent[e] = 1e-20                           # below the split's 2^-60 cut (hi = lo = 0)
    e = nxt(); ent[e] = ent[qt[0]]; ent[e, ::3] = np.float32(1e-40)   # subnormal values
    if nonfinite:
        e = nxt(); ent[e] = 1e38                        # products overflow: S' = inf, rescored
        e = nxt(); ent[e, 5] = np.nan
    return ent, rel, ent_im, rel_im, qh, qr, qt, qm


@pytest.mark.parametrize("wide", [None, "256", "128"])
@pytest.mark.parametrize("model,seed,nonfinite", [("distmult", 0, True), ("distmult", 1, False),
                                                  ("complex", 0, True), ("complex", 2, False)])
def test_mfma_filter_counts_equal_exact_sweep_and_oracle(oracle_mod, monkeypatch, model, seed, nonfinite, wide):
    """The split-bf16 MFMA filter (mmre_link_sweep_bf3): raw / filtered counts bit-equal to the
    score-storing exact sweep, to the exact count-only f32 MFMA sweep (MMRE_MFMA_FILTER=0) and to
    the oracle's Test.h restatement; the undecided list holds every truth and tie; entity slices
    sum to the whole table; a list too small for the undecided pairs (MMRE_BF3_CAP) takes the
    device-side fallback to the exact sweep with the same counts. wide: the wide sweep
    (k_sweep_bf3w, the default above 64 MB of planes: C5) forced at query tile 256 (500 queries:
    a padded last tile) or 128; every table here leaves the last entity tile partial."""
    import torch
    from mmre.link import FilterIndex, LinkSweep
    monkeypatch.setenv("MMRE_BF3_WIDE", "1" if wide else "0")
    if wide:
        monkeypatch.setenv("MMRE_BF3_QT", wide)
    ent, rel, ent_im, rel_im, qh, qr, qt, qm = _adversarial_dot(model, seed=seed, nonfinite=nonfinite,
                                                                Q=500 if wide == "256" else 300)
    E, R, d = ent.shape[0], rel.shape[0], rel.shape[1]
    rng = np.random.default_rng(seed + 10)
    fh, fr, ft = rng.integers(0, E, 3 * E), rng.integers(0, R, 3 * E), rng.integers(0, E, 3 * E)
    fh, fr, ft = np.concatenate([fh, qh]), np.concatenate([fr, qr]), np.concatenate([ft, qt])
    index = FilterIndex(fh, fr, ft, E, R)
    spec = _spec_from(model, ent, rel, ent_im, rel_im, dim=d)
    exact = _run(spec, qh, qr, qt, qm, index=index, scores=True)
    dev = spec.ent.device
    tq = lambda a, dt=np.int64: torch.from_numpy(np.asarray(a, dt)).to(dev)
    args = (tq(qh), tq(qr), tq(qt), tq(qm, np.int8))
    filt = tuple(torch.from_numpy(a).to(dev) for a in index.groups(qh, qr, qt, qm))

    def run(entity_range=None):
        sw = LinkSweep(spec)
        bufs = sw.alloc_queries(len(qh))
        f = filt if entity_range is None else tuple(
            torch.from_numpy(a).to(dev) for a in index.groups(qh, qr, qt, qm, entity_range=entity_range))
        res = sw.run(*args, filt=f, buffers=bufs, entity_range=entity_range)
        torch.cuda.synchronize()
        if model == "distmult" and os.environ.get("MMRE_MFMA_FILTER") != "0":
            # d = 48: the raw DistMult rows are split directly (mmre_link_sweep_bf3_rows) unless MMRE_BF3_RAW=0
            assert bufs["bf3_raw"] == (os.environ.get("MMRE_BF3_RAW") != "0")
        return res["counts"].cpu().numpy().copy(), sw.bf3_stats(bufs)

    fast, st = run()
    assert st is not None and not st["fallback"], st
    assert st["undecided"] >= len(qh), st               # every truth is listed (its S' is within the bound)
    assert np.array_equal(fast[:2], exact["counts"][:2])
    if model == "distmult":  # the prepared-copy path (k-major split + separate norms): the same counts
        monkeypatch.setenv("MMRE_BF3_RAW", "0")
        prep, st_prep = run()
        monkeypatch.delenv("MMRE_BF3_RAW")
        assert np.array_equal(prep, fast), (st_prep, st)  # (undecided pairs may differ: the norms round differently)
    monkeypatch.setenv("MMRE_MFMA_FILTER", "0")
    f32, st32 = run()
    monkeypatch.delenv("MMRE_MFMA_FILTER")
    assert st32 is None and np.array_equal(fast, f32)
    total = np.zeros_like(fast)
    for e0, e1 in ((0, 768), (768, 1664), (1664, E)):
        c, _ = run((e0, e1))
        total += c
    assert np.array_equal(total[:2], fast[:2])
    monkeypatch.setenv("MMRE_BF3_CAP", "64")
    small, st_small = run()
    monkeypatch.delenv("MMRE_BF3_CAP")
    assert st_small["fallback"], st_small
    assert np.array_equal(small, fast)
    hrt = oracle_mod.sorted_hrt(fh, fr, ft)
    for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
        sel = qm == mode_id
        o_pred = oracle_mod.link_predict(model, mode, ent, rel, qh[sel], qr[sel], qt[sel], ent_im=ent_im,
                                         rel_im=rel_im)
        o_c = oracle_mod.test_rank(mode, o_pred, qh[sel], qr[sel], qt[sel], hrt)
        assert np.array_equal(fast[:2, sel].T, o_c[:, :2])
    print(f"{model}: {st['undecided']} of {len(qh) * E} pairs rescored")


@pytest.mark.parametrize("model", ["distmult", "complex"])
def test_wide_sweep_lockstep_windows(oracle_mod, monkeypatch, model):
    """The wide split-bf16 sweep with its lock-step windows (MMRE_BF3_BLOCKED=1: BlockMap, the C5
    default above 64 MB of planes, which the small tables above never reach): counts bit-equal to
    the exact sweep, entity slices summing to the whole table."""
    import torch
    from mmre.link import FilterIndex, LinkSweep
    monkeypatch.setenv("MMRE_BF3_WIDE", "1")
    monkeypatch.setenv("MMRE_BF3_BLOCKED", "1")
    ent, rel, ent_im, rel_im, qh, qr, qt, qm = _adversarial_dot(model, E=4700, seed=3, nonfinite=False, Q=512)
    E, R, d = ent.shape[0], rel.shape[0], rel.shape[1]
    rng = np.random.default_rng(13)
    fh, fr, ft = rng.integers(0, E, 3 * E), rng.integers(0, R, 3 * E), rng.integers(0, E, 3 * E)
    fh, fr, ft = np.concatenate([fh, qh]), np.concatenate([fr, qr]), np.concatenate([ft, qt])
    index = FilterIndex(fh, fr, ft, E, R)
    spec = _spec_from(model, ent, rel, ent_im, rel_im, dim=d)
    exact = _run(spec, qh, qr, qt, qm, index=index, scores=True)
    dev = spec.ent.device
    tq = lambda a, dt=np.int64: torch.from_numpy(np.asarray(a, dt)).to(dev)
    args = (tq(qh), tq(qr), tq(qt), tq(qm, np.int8))

    def run(entity_range=None):
        sw = LinkSweep(spec)
        bufs = sw.alloc_queries(len(qh))
        f = tuple(torch.from_numpy(a).to(dev) for a in index.groups(qh, qr, qt, qm, entity_range=entity_range))
        res = sw.run(*args, filt=f, buffers=bufs, entity_range=entity_range)
        torch.cuda.synchronize()
        return res["counts"].cpu().numpy().copy(), sw.bf3_stats(bufs)

    fast, st = run()
    assert not st["fallback"] and st["undecided"] >= len(qh), st
    assert np.array_equal(fast[:2], exact["counts"][:2])
    total = np.zeros_like(fast)
    for e0, e1 in ((0, 2304), (2304, E)):
        c, _ = run((e0, e1))
        total += c
    assert np.array_equal(total[:2], fast[:2])
