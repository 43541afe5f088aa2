"""CPU-side tests: the C ABI library loads and exports every symbol of include/mmre.h, and the
host-side parts (metric reduction, glibc seeds, LCG bookkeeping, dataset/filter/train indices,
relation sharding) agree with the oracle and the reference's golden vectors. No GPU needed."""
import ctypes
import os
import sys
import re

import numpy as np
import pytest

from conftest import GOLDEN, REPO


def _header_functions():
    src = open(os.path.join(REPO, "include", "mmre.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mmre_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from mmre import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = _header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # every declared entry point is also bound (with argtypes) by the Python layer
    assert not [n for n in names if n not in _lib.SIGNATURES]


def test_product_binding_loads_without_gpu():
    from mmre import _lib
    L = _lib.lib()
    assert L.mmre_version() >= 100
    assert L.mmre_link_pad(1) == 128 and L.mmre_link_pad(129) == 256
    # VALU models pad d to 8 rows per plane, the MFMA models (DistMult/ComplEx) to 16 (one K stage)
    assert L.mmre_link_k(0, 200) == 200 and L.mmre_link_k(4, 13) == 32
    assert L.mmre_link_k(2, 200) == 208 and L.mmre_link_k(3, 200) == 400  # MFMA K: a multiple of 16


def test_metrics_host_matches_reference(golden):
    """mmre_link_metrics (host C++) reproduces Base.so's Test.h float accumulation bit-for-bit
    from the reference's own per-query counts."""
    from mmre.link import link_metrics
    g = golden("link_small")
    for name in ["transe", "transe_nonorm_margin", "transe_l2", "distmult", "complex", "rotate"]:
        for tc in (0, 1):
            h = g[f"{name}_tc{tc}_head_counts"].T.astype(np.int32)
            t = g[f"{name}_tc{tc}_tail_counts"].T.astype(np.int32)
            m = link_metrics(h, t)
            grp = m["filter_tc" if tc else "filter"]
            got = np.array([grp[k] for k in ("mrr", "mr", "hit10", "hit3", "hit1")], np.float32)
            assert np.array_equal(got, g[f"{name}_tc{tc}_metrics"]), (name, tc)


def test_metrics_host_matches_oracle_large():
    """Large counts (sums past 2^24, where float accumulation order matters)."""
    import oracle
    from mmre.link import link_metrics
    rng = np.random.default_rng(0)
    n = 40000
    h = rng.integers(0, 14000, (n, 4)).astype(np.int64)
    t = rng.integers(0, 14000, (n, 4)).astype(np.int64)
    o = oracle.link_metrics(h, t)
    m = link_metrics(h.T.astype(np.int32), t.T.astype(np.int32))
    for grp in ("filter", "raw", "filter_tc", "raw_tc"):
        for k in ("mrr", "mr", "hit10", "hit3", "hit1"):
            assert np.float32(m[grp][k]) == o[grp][k], (grp, k)


def test_glibc_seeds_and_lcg_advance(golden):
    import oracle
    from mmre.data import OpenKEDataset, TrainIndex
    from mmre.sampler import glibc_seeds
    assert glibc_seeds(5).tolist() == oracle.glibc_rand(5).tolist()
    assert glibc_seeds(3, skip=7).tolist() == oracle.glibc_rand(10)[7:].tolist()
    # mmre_sampler_advance == the oracle's sequential per-thread draws (and the reference's)
    g = golden("sampler_medium")
    d = OpenKEDataset(os.path.join(GOLDEN, "data", "medium"))
    from mmre._lib import call
    for name in sorted({k[:-len("_cfg")] for k in g if k.endswith("_cfg")}):
        threads, B, neg, negrel, mode, bern = g[f"{name}_cfg"].tolist()
        seeds = g[f"{name}_seeds0"].copy()
        for _ in range(3):
            call("mmre_sampler_advance", seeds.ctypes.data_as(ctypes.c_void_p), threads, B, neg, negrel, mode)
        assert np.array_equal(seeds, g[f"{name}_seeds_end"]), name


def test_train_index_matches_oracle():
    import oracle
    from mmre.data import OpenKEDataset, TrainIndex
    d = OpenKEDataset(os.path.join(GOLDEN, "data", "medium"))
    ix = TrainIndex(d.train[:, 0], d.train[:, 1], d.train[:, 2], d.n_ent, d.n_rel)
    o = oracle.train_index(d.train[:, 0], d.train[:, 1], d.train[:, 2], d.n_ent, d.n_rel)
    for a, b in [("train_list", "train_list"), ("head_hrt", "head"), ("tail_hrt", "tail"), ("rel_hrt", "rel"),
                 ("lef_head", "lef_head"), ("rig_head", "rig_head"), ("lef_tail", "lef_tail"),
                 ("rig_tail", "rig_tail"), ("lef_rel", "lef_rel"), ("rig_rel", "rig_rel")]:
        assert np.array_equal(getattr(ix, a), o[b]), a
    assert np.array_equal(ix.left_mean, o["left_mean"], equal_nan=True)
    assert np.array_equal(ix.right_mean, o["right_mean"], equal_nan=True)


def test_filter_index_and_type_masks():
    from mmre.data import OpenKEDataset
    from mmre.link import FilterIndex
    d = OpenKEDataset(os.path.join(GOLDEN, "data", "small"))
    idx = FilterIndex(*d.all_triples(), d.n_ent, d.n_rel, d.type_heads, d.type_tails)
    h, r, t = d.test_list()
    n = len(h)
    qh, qr, qt = (np.concatenate([x, x]) for x in (h, r, t))
    qm = np.r_[np.zeros(n, np.int8), np.ones(n, np.int8)]
    off, ids = idx.filters(qh, qr, qt, qm)
    S = set(zip(*(x.tolist() for x in d.all_triples())))
    for i in range(2 * n):
        got = set(ids[off[i]:off[i + 1]].tolist())
        if qm[i] == 0:
            exp = {j for j in range(d.n_ent) if (j, qr[i], qt[i]) in S}
        else:
            exp = {j for j in range(d.n_ent) if (qh[i], qr[i], j) in S}
        assert got == exp and off[i + 1] - off[i] == len(exp)
    mh, mt = idx.type_masks()
    for r_ in range(d.n_rel):
        bits = [(mh[r_, e >> 5] >> (e & 31)) & 1 for e in range(d.n_ent)]
        assert np.nonzero(bits)[0].tolist() == d.type_heads[r_]
        bits = [(mt[r_, e >> 5] >> (e & 31)) & 1 for e in range(d.n_ent)]
        assert np.nonzero(bits)[0].tolist() == d.type_tails[r_]


def test_filter_groups_partition():
    """FilterIndex.groups: a partition of the queries into (mode, r, anchor) groups whose
    shared list equals every member's own filter list."""
    from mmre.data import OpenKEDataset
    from mmre.link import FilterIndex
    d = OpenKEDataset(os.path.join(GOLDEN, "data", "medium"))
    idx = FilterIndex(*d.all_triples(), d.n_ent, d.n_rel)
    h, r, t = d.test_list()
    n = len(h)
    qh, qr, qt = (np.concatenate([x, x]) for x in (h, r, t))
    qm = np.r_[np.zeros(n, np.int8), np.ones(n, np.int8)]
    off, ids = idx.filters(qh, qr, qt, qm)
    gqo, gq, goff, gids, entry_q = idx.groups(qh, qr, qt, qm, max_group=3)
    assert len(entry_q) == len(gids)
    assert gqo[0] == 0 and gqo[-1] == 2 * n and np.all(np.diff(gqo) > 0) and np.all(np.diff(gqo) <= 3)
    assert np.array_equal(np.sort(gq), np.arange(2 * n))
    assert len(goff) == len(gqo) and goff[-1] == len(gids)
    for g in range(len(gqo) - 1):
        members = gq[gqo[g]:gqo[g + 1]]
        lst = gids[goff[g]:goff[g + 1]].tolist()
        m0 = members[0]
        assert np.all(entry_q[goff[g]:goff[g + 1]] == m0)
        for q in members:
            assert qm[q] == qm[m0] and qr[q] == qr[m0]
            assert (qt[q] == qt[m0]) if qm[q] == 0 else (qh[q] == qh[m0])
            assert ids[off[q]:off[q + 1]].tolist() == lst
    assert len(gqo) - 1 < 2 * n  # the synthetic test set shares keys


def test_test_list_order_matches_reference(golden):
    """testList sorted by (r, h, t) (Reader.h:227): the reference Base.so's query order."""
    from mmre.data import OpenKEDataset
    g = golden("link_small")
    h, r, t = OpenKEDataset(os.path.join(GOLDEN, "data", "small")).test_list()
    assert np.array_equal(h, g["qh"]) and np.array_equal(r, g["qr"]) and np.array_equal(t, g["qt"])


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_lpt_partition(world):
    from mmre.data import load_zs_test
    from mmre.sharding import lpt_partition
    z = load_zs_test("FB15K-237-ZS")
    qr = np.concatenate([z["r"], z["r"]])
    masks = lpt_partition(qr, world, split=False)
    assert np.array_equal(np.sum(masks, 0), np.ones(len(qr)))  # a partition
    for m in masks:  # whole relations per rank
        for r in np.unique(qr[m]):
            assert m[qr == r].all()
    loads = [m.sum() for m in masks]
    # FB15K-237-ZS LPT ceilings 1.99 / 3.98 / 7.84 at 2 / 4 / 8 ranks
    ceiling = len(qr) / max(loads)
    assert ceiling >= {1: 1.0, 2: 1.98, 4: 3.9, 8: 7.5}[world]


@pytest.mark.parametrize("dataset", ["FB15K-237-ZS", "DB15K-ZS"])
@pytest.mark.parametrize("world", [2, 3, 8, 16])
def test_lpt_partition_with_query_pieces(dataset, world):
    """SURVEY §8(e) fallback: relations above the per-rank share are cut into contiguous
    query pieces; DB15K-ZS's whole-relation ceiling at 8 ranks (5.41x) rises to > 7.5x, and
    every rank's share of a relation is a run of consecutive queries of it (Test.h order)."""
    from mmre.data import load_zs_test
    from mmre.sharding import lpt_partition
    z = load_zs_test(dataset)
    qr = np.concatenate([z["r"], z["r"]])
    masks = lpt_partition(qr, world)
    assert np.array_equal(np.sum(masks, 0), np.ones(len(qr)))
    ceiling = len(qr) / max(m.sum() for m in masks)
    assert ceiling >= 0.93 * world
    whole = len(qr) / max(m.sum() for m in lpt_partition(qr, world, split=False))
    assert ceiling >= whole - 1e-9
    for m in masks:
        for r in np.unique(qr[m]):
            idx = np.nonzero(qr == r)[0]          # the relation's queries in order
            mine = np.nonzero(m[idx])[0]          # positions of this rank's among them
            # pieces are contiguous in the relation's own order: few runs
            runs = 1 + int(np.sum(np.diff(mine) > 1))
            assert runs <= -(-len(idx) // -(-len(qr) // world)) + 1
    if dataset == "DB15K-ZS" and world == 8:
        assert whole < 5.5 and ceiling > 7.5


def test_zs_datasets_shipped():
    from mmre.data import load_zs_test
    z = load_zs_test("FB15K-237-ZS")
    assert len(z["h"]) == 17596 and int(z["n_ent"]) == 14208 and int(z["n_rel"]) == 235
    assert len(np.unique(z["r"])) == 29
    z = load_zs_test("DB15K-ZS")
    assert len(z["h"]) == 5653 and int(z["n_ent"]) == 12741 and int(z["n_rel"]) == 157


def test_entity_slices_and_restricted_filter_lists():
    """Entity sharding's host side: slices cut at whole 128-entity tiles cover the table once,
    and filter lists restricted to each slice partition the whole list of every group (same
    scoring member per entry)."""
    from mmre.link import FilterIndex
    from mmre.sharding import entity_slices
    for E, W in ((14541, 8), (300, 4), (100, 3), (129, 2)):
        sl = entity_slices(E, W)
        assert sl[0][0] == 0 and sl[-1][1] == E
        assert all(a % 128 == 0 and a <= b for a, b in sl)
        assert all(sl[k][1] == sl[k + 1][0] for k in range(W - 1))
    rng = np.random.default_rng(0)
    E, R = 500, 7
    h, r, t = rng.integers(0, E, 3000), rng.integers(0, R, 3000), rng.integers(0, E, 3000)
    ix = FilterIndex(h, r, t, E, R)
    qm = np.r_[np.zeros(100, np.int8), np.ones(100, np.int8)]
    full = ix.groups(h[:200], r[:200], t[:200], qm)
    parts = [ix.groups(h[:200], r[:200], t[:200], qm, entity_range=s) for s in entity_slices(E, 3)]
    for g in range(len(full[0]) - 1):
        whole = full[3][full[2][g]:full[2][g + 1]]
        got = np.concatenate([p[3][p[2][g]:p[2][g + 1]] for p in parts])
        assert sorted(got.tolist()) == sorted(whole.tolist())
        for p, (e0, e1) in zip(parts, entity_slices(E, 3)):
            ids = p[3][p[2][g]:p[2][g + 1]]
            assert np.all((ids >= e0) & (ids < e1))
            assert np.all(p[4][p[2][g]:p[2][g + 1]] == full[0][g] * 0 + full[1][full[0][g]])


def test_sgd_routes_only_plain_cuda_steps_to_hip():
    """mmre.optim.SGD is torch.optim.SGD wherever the HIP step does not apply (host tensors,
    momentum, weight decay): bit-identical to torch there; the eligibility test itself."""
    import torch
    from mmre.optim import SGD
    g = torch.Generator().manual_seed(0)
    for kw in ({}, {"momentum": 0.9}, {"weight_decay": 0.01}, {"momentum": 0.5, "nesterov": True}):
        a = [torch.randn(37, 5, generator=g), torch.randn(11, generator=g)]
        b = [x.clone() for x in a]
        for ps in (a, b):
            for p in ps:
                p.grad = torch.ones_like(p) * 0.25
        torch.optim.SGD(a, lr=0.3, **kw).step()
        SGD(b, lr=0.3, **kw).step()
        assert all(torch.equal(x, y) for x, y in zip(a, b)), kw
    opt = SGD([torch.zeros(3, requires_grad=True)], lr=0.1)
    assert opt._plain(opt.param_groups[0])
    assert not opt._plain(dict(opt.param_groups[0], momentum=0.9))
    assert not opt._plain(dict(opt.param_groups[0], weight_decay=1e-4))


def test_sgd_closure_runs_first_and_fallbacks_are_counted():
    """step(closure) runs the closure before choosing the parameters (a parameter
    whose .grad the closure creates is updated, as torch.optim.SGD does), and every step that
    takes torch's path is counted with its reason."""
    import torch
    from mmre.optim import SGD
    p = torch.ones(4, requires_grad=True)
    q = torch.ones(4, requires_grad=True)
    opt = SGD([p], lr=0.5)
    ref = torch.optim.SGD([q], lr=0.5)
    before = SGD.fallback_steps

    def closure(x):
        def f():
            x.grad = None
            loss = (x * x).sum()
            loss.backward()
            return loss
        return f

    opt.step(closure(p))
    ref.step(closure(q))
    assert torch.equal(p, q) and not torch.equal(p, torch.ones(4))
    assert SGD.fallback_steps == before + 1 and "device" in SGD.fallback_reason


def test_import_prob_is_the_reference(golden):
    """mmre_import_prob (host, Reader.h:26-49) reproduces the reference Base.so's `prob` table bit
    for bit at every fixture temperature (tests/golden/make_sampler_p.py)."""
    from mmre._lib import call
    g = golden("sampler_p")
    path = os.path.join(GOLDEN, "data", "prel", "kl_prob.txt")
    n_rel = int(open(os.path.join(GOLDEN, "data", "prel", "relation2id.txt")).readline())
    for name in sorted(k[:-len("_temp")] for k in g if k.endswith("_temp")):
        out = np.zeros((n_rel, n_rel - 1), np.float32)
        call("mmre_import_prob", path.encode(), n_rel, float(g[f"{name}_temp"]), out.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(out.ravel(), g[f"{name}_prob"]), name
    with pytest.raises(Exception):
        call("mmre_import_prob", b"/nonexistent/kl_prob.txt", n_rel, 1.0, out.ctypes.data_as(ctypes.c_void_p))


def test_import_prob_wide_table_is_the_reference(golden, tmp_path):
    """200 relations, KL values over [0, 20), temperatures 0.1-2: exp(-x / T) spans many binades,
    so evaluating Reader.h:40's unqualified exp(float) as expf instead of libstdc++'s
    (float)exp((double)x) would differ by an ulp somewhere. Bit-equal to the
    reference Base.so's `prob` table, and so is the oracle's restatement."""
    import oracle as oracle_mod
    from mmre._lib import call
    sys.path.insert(0, os.path.join(GOLDEN))
    from make_sampler_p import WIDE_REL, WIDE_TEMPS, wide_kl_text
    g = golden("sampler_p")
    path = tmp_path / "kl_prob.txt"
    path.write_text(wide_kl_text())
    for T in WIDE_TEMPS:
        want = g[f"wide_prob_T{T}"]
        out = np.zeros((WIDE_REL, WIDE_REL - 1), np.float32)
        call("mmre_import_prob", str(path).encode(), WIDE_REL, float(T), out.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(out.ravel(), want), T
        assert np.array_equal(np.asarray(oracle_mod.import_prob(str(path), WIDE_REL, T)).ravel(), want), T


def test_bench_quotes_pmc_traffic_only_for_this_build(tmp_path, monkeypatch):
    """bench.py reads roofline.traffic from profiles/pmc_<config>.json only when the summary's
    __build__.lib_sha256 is the loaded library's; any other build's counters give None and a reason."""
    import json as _json
    import bench
    from mmre._lib import lib_identity
    mine = lib_identity()["sha256"]
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    k = bench.KERNEL_NAMES["transe"]
    for sha, want in ((mine, (2 * 100.0 + 50.0) * 1024.0), ("0123456789abcdef", None)):
        (prof / "pmc_c2.json").write_text(_json.dumps({
            "__build__": {"lib_sha256": sha},
            f"void mmre::{k}(float const*)": {"FETCH_SIZE": 100.0, "WRITE_SIZE": 50.0}}))
        got, src = bench.pmc_traffic("c2", "transe")
        assert got == want, (sha, got, src)
        if want is None:
            assert "not this build" in src
    (prof / "pmc_ns.json").write_text(_json.dumps({
        "__build__": {"lib_sha256": mine},
        "mmre::k_ns_prepass(x)": {"FETCH_SIZE": 1.0, "WRITE_SIZE": 1.0},
        "void mmre::k_ns_transe_fused<4, false>(x)": {"FETCH_SIZE": 2.0, "WRITE_SIZE": 1.0}}))
    tot, src, per = bench.pmc_step_traffic("ns", ["k_ns_prepass(", "k_ns_transe_fused<4, false>"])
    assert tot == (3.0 + 5.0) * 1024.0 and len(per) == 2
    assert bench.pmc_step_traffic("ns", ["k_ns_row_owner"])[0] is None


@pytest.mark.parametrize("world", [2, 4, 8])
def test_lpt_partition_weighted(world):
    """Cost-aware packing: with per-query weights the ranks' weight loads
    are balanced to within one query piece, pieces stay contiguous runs of a relation, and
    uniform weights reproduce the count-based partition's balance."""
    from mmre.data import load_zs_test
    from mmre.sharding import cost_weights, lpt_partition
    z = load_zs_test("FB15K-237-ZS")
    qr = np.concatenate([z["r"], z["r"]])
    rng = np.random.default_rng(world)
    und = np.where(rng.random(len(qr)) < 0.05, rng.integers(100, 3000, len(qr)), rng.integers(0, 40, len(qr)))
    und[qr == np.bincount(qr).argmax()] *= 10       # one relation's queries are costly
    w = cost_weights(und, 14208)
    masks = lpt_partition(qr, world, weights=w)
    assert np.array_equal(np.sum(masks, 0), np.ones(len(qr)))
    loads = np.array([w[m].sum() for m in masks])
    assert loads.max() <= w.sum() / world + w.max() + 1e-6
    for m in masks:
        for r in np.unique(qr[m]):
            idx = np.nonzero(qr == r)[0]
            mine = np.nonzero(m[idx])[0]
            assert 1 + int(np.sum(np.diff(mine) > 1)) <= world + 1
    u = lpt_partition(qr, world, weights=np.ones(len(qr)))
    assert len(qr) / max(m.sum() for m in u) >= 0.93 * world
