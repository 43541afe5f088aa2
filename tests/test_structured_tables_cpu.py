"""CPU checks of the reference-rank fixtures (tests/golden/ref_parity_<config>.npz, made by
tests/golden/make_ref_parity.py from the reference's Base.so Tester loop) and of the structured
tables behind them (mmre.workloads.structured_tables):

* the tables rebuilt in this process hash to the fixture's sha256 (the construction is
  deterministic; tests/test_ref_fixture_gpu.py repeats the check on the GPU box);
* the fixture is non-degenerate: filtered hit@10 well above 0, and truths at every rank boundary;
* the build's host Test.h reduction (mmre_link_metrics, P14 order) of the reference's own
  per-query counts gives Base.so's getTestLink* values bit for bit -- so GPU counts equal to the
  reference's imply bit-equal metrics;
* near lists are well formed (sorted sweeps, ids in range, truth excluded).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5"])
def test_ref_parity_fixture(config, golden):
    from mmre.link import link_metrics
    from mmre.workloads import REF_PARITY, TRAINED_TABLES, ref_parity_workload, tables_sha256, zs_workload
    fx = golden(f"ref_parity_{config}")
    if config in TRAINED_TABLES:
        # trained tables (C2): rebuilt only on a GPU (tests/test_ref_fixture_gpu.py checks their
        # sha256 there); here the workload's queries and the fixture itself
        (dataset, model, dim), _, _ = REF_PARITY[config]
        w = zs_workload(dataset, model, dim)
        assert len(str(fx["tables_sha256"])) == 64
    else:
        w = ref_parity_workload(config)
        assert tables_sha256(w) == str(fx["tables_sha256"])
    n = len(w["test_h"])
    assert REF_PARITY[config][1] in (None, n)
    assert np.array_equal(fx["q"], np.stack([w["test_h"], w["test_r"], w["test_t"]], 1))
    c = fx["counts"].astype(np.int32)                      # (2, n, 2)
    E = int(fx["n_ent"])
    assert np.all(c[:, :, 1] <= c[:, :, 0]) and np.all(c >= 0) and np.all(c <= E - 1)
    filt = c[:, :, 1].reshape(-1)
    assert np.mean(filt < 10) > 0.4 and np.mean(filt < 1) > 0.2
    for k in (0, 1, 2, 3, 9, 10):                           # truths on both sides of every hit@k edge
        assert np.any(filt == k)
    z = np.zeros((2, n), np.int32)
    head = np.concatenate([c[0].T[[0, 1]], z])             # (4, n) raw, filt, raw_tc, filt_tc
    tail = np.concatenate([c[1].T[[0, 1]], z])
    m = link_metrics(head, tail)["filter"]
    got = np.array([m["mrr"], m["mr"], m["hit10"], m["hit3"], m["hit1"]], np.float32)
    assert np.array_equal(got.view(np.uint32), fx["metrics"].astype(np.float32).view(np.uint32))
    off, ids = fx["near_off"], fx["near_ids"]
    assert off[0] == 0 and off[-1] == len(ids) == len(fx["near_scores"]) and np.all(np.diff(off) >= 0)
    assert len(off) == 2 * n + 1 and np.all((ids >= 0) & (ids < E))
    sweep = np.repeat(np.arange(2 * n), np.diff(off))
    truth = np.r_[w["test_h"], w["test_t"]]
    assert not np.any(ids == truth[sweep])
