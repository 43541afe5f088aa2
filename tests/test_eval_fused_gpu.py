"""The fused TransE L1 evaluation (mmre_link_evaluate_l1q, csrc/link.hip K1-K3 + the gated sweeps):
one C-ABI call doing entity prep, query prep, truth scores, filter-list scores and counts, the
L1 filter's quantization and probe and the sweep, with independent work fused into shared
launches. Bar: everything it leaves in HBM -- the entity and query planes and rows, truth scores,
counts -- bit-identical to the separate entry points (mmre_link_prepare_entities /
_prepare_queries / _truth_grouped / _sweep_l1q, MMRE_FUSED_EVAL=0), and counts equal to the
oracle's Test.h restatement (TransE.py:46-60, Test.h:65-192); every code width; entity slices;
repeated calls and hipGraph replays (the grid tickets reset themselves)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from test_sweep_filters_gpu import _adversarial
from test_link_gpu import _spec_from

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _eval(spec, qh, qr, qt, qm, index, fused, monkeypatch, entity_range=None, reps=1, graph=False):
    from mmre.link import LinkSweep
    monkeypatch.setenv("MMRE_FUSED_EVAL", "1" if fused else "0")
    to = lambda a, dt=np.int64: torch.from_numpy(np.asarray(a, dt)).to(DEV)
    filt = tuple(torch.from_numpy(a).to(DEV) for a in index.groups(qh, qr, qt, qm, entity_range=entity_range))
    sw = LinkSweep(spec)
    assert sw.fused_eval == fused
    bufs = sw.alloc_queries(len(qh))
    args = (to(qh), to(qr), to(qt), to(qm, np.int8))
    for _ in range(reps):
        sw.run(*args, filt=filt, buffers=bufs, entity_range=entity_range)
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            sw.run(*args, filt=filt, buffers=bufs, entity_range=entity_range)
        for _ in range(3):
            bufs["counts"].fill_(-7)
            g.replay()
    torch.cuda.synchronize()
    st = sw.l1q_stats(bufs)
    n = len(qh)
    out = {"counts": bufs["counts"].cpu().numpy().copy(), "truth": bufs["truth"].cpu().numpy().copy(),
           "q_km": bufs["q_km"].cpu().numpy().copy(), "q_rows": bufs["q_rows"][:n].cpu().numpy().copy(),
           "q_true": bufs["q_true"][:n].cpu().numpy().copy(), "ent_km": sw.ent_km.cpu().numpy().copy(),
           "ent_rows": sw.ent_rows.cpu().numpy().copy(), "st": st}
    monkeypatch.delenv("MMRE_FUSED_EVAL")
    return out


def _same(a, b):
    for k in ("counts", "truth", "q_km", "q_rows", "q_true", "ent_km", "ent_rows"):
        x, y = a[k], b[k]
        assert np.array_equal(x.view(np.uint32) if x.dtype == np.float32 else x,
                              y.view(np.uint32) if y.dtype == np.float32 else y), k
    sa, sb = a["st"], b["st"]
    assert sa["bits"] == sb["bits"] and sa["fallback"] == sb["fallback"], (sa, sb)
    assert sa["undecided"] == sb["undecided"], (sa, sb)
    assert sa["guarded"] == 0 and sb["guarded"] == 0


@pytest.mark.parametrize("norm", [True, False])
@pytest.mark.parametrize("bits", [None, "8", "16"])
def test_fused_equals_separate_adversarial(oracle_mod, monkeypatch, norm, bits):
    from mmre.link import FilterIndex
    if bits is None:
        monkeypatch.delenv("MMRE_L1_BITS", raising=False)
    else:
        monkeypatch.setenv("MMRE_L1_BITS", bits)
    ent, rel, qh, qr, qt, qm = _adversarial(E=2100, d=40, Q=300, seed=3, model="transe", huge=False)
    E, R = ent.shape[0], rel.shape[0]
    rng = np.random.default_rng(7)
    fh, fr, ft = rng.integers(0, E, 3 * E), rng.integers(0, R, 3 * E), rng.integers(0, E, 3 * E)
    fh, fr, ft = np.r_[fh, qh], np.r_[fr, qr], np.r_[ft, qt]
    index = FilterIndex(fh, fr, ft, E, R)
    spec = _spec_from("transe", ent, rel, dim=40, norm=norm)
    fused = _eval(spec, qh, qr, qt, qm, index, True, monkeypatch, reps=2)
    sep = _eval(spec, qh, qr, qt, qm, index, False, monkeypatch)
    _same(fused, sep)
    hrt = oracle_mod.sorted_hrt(fh, fr, ft)
    for mode_id, mode in ((0, "head_batch"), (1, "tail_batch")):
        sel = qm == mode_id
        o_pred = oracle_mod.link_predict("transe", mode, ent, rel, qh[sel], qr[sel], qt[sel], norm_flag=norm)
        o_c = oracle_mod.test_rank(mode, o_pred, qh[sel], qr[sel], qt[sel], hrt)
        assert np.array_equal(fused["counts"][:2, sel].T, o_c[:, :2])


def test_fused_huge_values_take_the_f32_fallback(monkeypatch):
    """A row of 3e19 and a NaN make M non-finite: K1's last block picks the f32 sweep."""
    from mmre.link import FilterIndex
    ent, rel, qh, qr, qt, qm = _adversarial(E=1500, d=48, Q=257, seed=2, model="transe", huge=True)
    E, R = ent.shape[0], rel.shape[0]
    index = FilterIndex(qh, qr, qt, E, R)
    spec = _spec_from("transe", ent, rel, dim=48, norm=False)
    fused = _eval(spec, qh, qr, qt, qm, index, True, monkeypatch)
    sep = _eval(spec, qh, qr, qt, qm, index, False, monkeypatch)
    assert fused["st"]["fallback"], fused["st"]
    for k in ("counts", "q_km", "ent_km"):
        assert np.array_equal(fused[k].view(np.uint32) if fused[k].dtype == np.float32 else fused[k],
                              sep[k].view(np.uint32) if sep[k].dtype == np.float32 else sep[k]), k
    t1, t2 = fused["truth"], sep["truth"]
    assert np.array_equal(np.isnan(t1), np.isnan(t2)) and np.array_equal(t1[~np.isnan(t1)], t2[~np.isnan(t2)])


def test_fused_c2_slices_graph_and_repeats(monkeypatch):
    """C2 (FB15K-237-ZS TransE d=200, xavier tables: the probe picks the 16-bit codes; and
    the 8-bit codes forced): fused == separate, entity slices sum to the whole table, graph
    replays and repeated calls give the same counts."""
    from mmre.link import FilterIndex, HEAD, TAIL, ScoreSpec
    from mmre.workloads import zs_workload
    w = zs_workload("FB15K-237-ZS", "transe", 200)
    n, E = len(w["test_h"]), w["n_ent"]
    qh, qr, qt = (np.r_[w[k], w[k]] for k in ("test_h", "test_r", "test_t"))
    qm = np.r_[np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)]
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], E, w["n_rel"])
    spec = ScoreSpec(model="transe", ent=w["ent"].to(DEV), rel=w["rel"].to(DEV), dim=200, norm_flag=True, pred_kind=0)
    fused = _eval(spec, qh, qr, qt, qm, index, True, monkeypatch, reps=3, graph=True)
    sep = _eval(spec, qh, qr, qt, qm, index, False, monkeypatch)
    _same(fused, sep)
    # forced 8-bit codes on these tables put ~16 % of the pairs in the band (all rescored)
    monkeypatch.setenv("MMRE_L1_BITS", "8")
    f8 = _eval(spec, qh, qr, qt, qm, index, True, monkeypatch)
    s8 = _eval(spec, qh, qr, qt, qm, index, False, monkeypatch)
    monkeypatch.delenv("MMRE_L1_BITS")
    _same(f8, s8)
    assert np.array_equal(f8["counts"], fused["counts"])
    print(f"C2 forced 8-bit: {f8['st']}")
    total = np.zeros_like(fused["counts"])
    for e0, e1 in ((0, 4096), (4096, 9984), (9984, E)):
        part = _eval(spec, qh, qr, qt, qm, index, True, monkeypatch, entity_range=(e0, e1))
        sep_part = _eval(spec, qh, qr, qt, qm, index, False, monkeypatch, entity_range=(e0, e1))
        assert np.array_equal(part["counts"], sep_part["counts"])
        total += part["counts"]
    assert np.array_equal(total, fused["counts"])
    print(f"C2 fused: {fused['st']}")
