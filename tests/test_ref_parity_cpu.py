"""bench.py's cpu_baseline / parity leg on CPU: oracle/ref_tester.py runs the reference's Tester
loop (reference Base.so + the reference predict op sequences) on a workload, and
bench.parity_block compares per-query counts with a count table laid out like the GPU
evaluation's -- here the oracle's, so the comparison machinery itself is checked without a GPU."""
import os

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(REPO, "oracle", "_ref", "Base.so")

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref/Base.so not built")


def _workload(model, n_ent=300, n_rel=7, n_test=60, n_train=2000, dim=24, seed=0):
    from mmre.data import sorted_rel2
    rng = np.random.default_rng(seed)
    h, r, t = rng.integers(0, n_ent, n_test), rng.integers(0, n_rel, n_test), rng.integers(0, n_ent, n_test)
    th, tr, tt = sorted_rel2(np.stack([h, t, r], 1))
    g = torch.Generator().manual_seed(seed)
    w = dict(dataset="synthetic", model=model, dim=dim, n_ent=n_ent, n_rel=n_rel, test_h=th, test_r=tr, test_t=tt,
             norm_flag=model == "transe")
    if model == "rotate":
        w["margin"], w["epsilon"] = 6.0, 2.0
        w["ent"] = torch.rand((n_ent, 2 * dim), generator=g) - 0.5
        w["rel"] = torch.rand((n_rel, dim), generator=g) - 0.5
    else:
        w["ent"], w["rel"] = torch.rand((n_ent, dim), generator=g) - 0.5, torch.rand((n_rel, dim), generator=g) - 0.5
    if model == "complex":
        w["ent_im"], w["rel_im"] = torch.rand((n_ent, dim), generator=g) - 0.5, torch.rand((n_rel, dim), generator=g) - 0.5
    fh, fr, ft = rng.integers(0, n_ent, n_train), rng.integers(0, n_rel, n_train), rng.integers(0, n_ent, n_train)
    w["filter_h"], w["filter_r"], w["filter_t"] = (np.concatenate([a, b]) for a, b in ((fh, th), (fr, tr), (ft, tt)))
    return w


def _oracle_counts(oracle_mod, w, types=False):
    kw = {}
    if w["model"] == "transe":
        kw = dict(norm_flag=True)
    elif w["model"] == "rotate":
        kw = dict(margin=6.0, phase_denom=oracle_mod.rotate_phase_denom(6.0, 2.0, w["dim"]))
    ent, rel = w["ent"].numpy(), w["rel"].numpy()
    ei = w["ent_im"].numpy() if "ent_im" in w else None
    ri = w["rel_im"].numpy() if "rel_im" in w else None
    hrt = oracle_mod.sorted_hrt(w["filter_h"], w["filter_r"], w["filter_t"])
    out, scores = [], []
    for mode in ("head_batch", "tail_batch"):
        p = oracle_mod.link_predict(w["model"], mode, ent, rel, w["test_h"], w["test_r"], w["test_t"], ent_im=ei,
                                    rel_im=ri, **kw)
        tk = {}
        if types:  # CSR per relation (Test.h's head_type / tail_type ranges, sorted)
            lists = w["type_heads" if mode == "head_batch" else "type_tails"]
            tk = dict(type_off=np.r_[0, np.cumsum([len(x) for x in lists])],
                      type_ids=np.concatenate([np.sort(np.asarray(x, np.int64)) for x in lists]))
        out.append(oracle_mod.test_rank(mode, p, w["test_h"], w["test_r"], w["test_t"], hrt, **tk).T)
        scores.append(p)
    # (4, 2n) counts: head block then tail block; the oracle's scores are the GPU's bit for bit
    return np.concatenate(out, 1).astype(np.int32), scores


@pytest.mark.parametrize("model", ["transe", "distmult", "complex", "rotate"])
@pytest.mark.parametrize("n_sample", [60, 25])
def test_ref_leg_and_parity_block(oracle_mod, model, n_sample):
    import bench
    w = _workload(model)
    counts, sc = _oracle_counts(oracle_mod, w)
    ref = bench.ref_tester_leg(w, n_sample, reps=2)
    assert ref is not None
    assert ref["counts"].shape == (2, n_sample, 2)
    assert len(ref["elapsed_reps"]) == 2
    par = bench.parity_block(ref, counts, len(w["test_h"]), w,
                             torch.from_numpy(np.concatenate([sc[0][:n_sample], sc[1][:n_sample]])))
    assert par["window_ok"], par   # the measured error is far inside the near-tie window
    assert par["queries_match"] and par["sweeps"] == 2 * n_sample
    assert ref["threads"] >= 1 and len(ref["chunk_n"]) == ref["threads"]
    # the oracle's canonical arithmetic differs from the reference's torch order only inside near ties
    assert par["unexplained_mismatches"] == 0, par
    if par["filt_mismatches"] == 0:
        assert par["metrics_bit_equal"], par   # Test.h reduction of equal counts: bit-identical metrics
    cpu = bench.cpu_baseline_block(ref, w)
    assert cpu["kind"] == "reference" and cpu["value"] > 0
    assert cpu["value_min"] <= cpu["value"] <= cpu["value_max"] and cpu["reps"] == 2


def test_parity_block_reports_a_planted_mismatch(oracle_mod):
    import bench
    w = _workload("distmult")
    counts, sc = _oracle_counts(oracle_mod, w)
    ref = bench.ref_tester_leg(w, 60, reps=1)
    bad = counts.copy()
    bad[1, 3] += 5     # filtered head count of query 3
    bad[0, 60 + 7] += 2  # raw tail count of query 7
    par = bench.parity_block(ref, bad, 60, w, torch.from_numpy(np.concatenate(sc)))
    assert par["filt_mismatches"] >= 1 and par["raw_mismatches"] >= 1
    assert par["unexplained_mismatches"] >= 1
    assert not par["metrics_bit_equal"]


@pytest.mark.parametrize("model", ["transe", "distmult"])
def test_ref_leg_type_constrained(oracle_mod, model):
    """The type-constrained leg (bench.py --type-constrain): ref_tester writes type_constrain.txt
    (Reader.h:267-317's format), runs testHead / testTail with type_constrain and reads Base.so's
    *_constrain counters; they equal the oracle's Test.h restatement, and parity_block(tc=True)
    compares the constrained columns."""
    import bench
    w = _workload(model)
    rng = np.random.default_rng(5)
    n_ent, n_rel = w["n_ent"], w["n_rel"]
    # per relation: the heads / tails of its known triples (n-n.py's rule) plus random extras
    fh, fr, ft = (np.asarray(w[k]) for k in ("filter_h", "filter_r", "filter_t"))
    w["type_heads"] = [np.unique(np.r_[fh[fr == r], rng.integers(0, n_ent, 20)]) for r in range(n_rel)]
    w["type_tails"] = [np.unique(np.r_[ft[fr == r], rng.integers(0, n_ent, 20)]) for r in range(n_rel)]
    counts, sc = _oracle_counts(oracle_mod, w, types=True)
    ref = bench.ref_tester_leg(w, 40, reps=1)
    assert ref is not None and ref["counts"].shape == (2, 40, 4)
    par = bench.parity_block(ref, counts, len(w["test_h"]), w,
                             torch.from_numpy(np.concatenate([sc[0][:40], sc[1][:40]])), tc=True)
    assert par["window_ok"] and par["unexplained_mismatches"] == 0, par
    if par["filt_mismatches"] == 0:
        assert par["metrics_bit_equal"], par
    # the constrained counts are not the unconstrained ones (the types exclude entities)
    assert (ref["counts"][:, :, 2] <= ref["counts"][:, :, 0]).all()
    assert (ref["counts"][:, :, 2] < ref["counts"][:, :, 0]).any()


def test_ref_trainer_leg_reports_its_spread():
    """The NS line's cpu_baseline: the reference training leg repeated; the reported value is the
    median repetition's rate and lies inside the min / max of that same statistic."""
    import bench
    w = _workload("transe")
    cpu = bench.ref_trainer_leg(w, 64, 4, 5.0, steps=2, reps=3)
    assert cpu is not None and cpu["kind"] == "reference" and cpu["reps"] == 3
    assert cpu["value_min"] <= cpu["value"] <= cpu["value_max"]
    assert cpu["value"] == cpu["value_median"]
