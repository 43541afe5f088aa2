"""Pin the oracle (oracle/) against golden vectors produced by the reference itself
(tests/golden/make_golden.py: reference OpenKE models + reference Base.so + repo modules)."""
import numpy as np
import pytest

LINK_MODELS = [
    # fixture name, oracle model, mode-independent kwargs builder
    ("transe", "transe"), ("transe_nonorm_margin", "transe"), ("transe_l2", "transe_l2"),
    ("distmult", "distmult"), ("complex", "complex"), ("rotate", "rotate"),
]


def _tables(g, name):
    if name == "complex":
        return (g[f"{name}.ent_re_embeddings.weight"], g[f"{name}.rel_re_embeddings.weight"],
                g[f"{name}.ent_im_embeddings.weight"], g[f"{name}.rel_im_embeddings.weight"])
    return g[f"{name}.ent_embeddings.weight"], g[f"{name}.rel_embeddings.weight"], None, None


def _kw(name, oracle_mod):
    if name == "transe":
        return dict(norm_flag=True)
    if name == "transe_nonorm_margin":
        return dict(norm_flag=False, margin=5.0)
    if name == "transe_l2":
        return dict(norm_flag=True)
    if name == "rotate":
        return dict(margin=6.0, phase_denom=oracle_mod.rotate_phase_denom(6.0, 2.0, 16))
    return {}


def _score_tol(ref):
    return 1e-4 * np.maximum(1.0, np.abs(ref))


@pytest.mark.parametrize("name,model", LINK_MODELS)
@pytest.mark.parametrize("mode", ["head_batch", "tail_batch"])
def test_link_scores_match_reference(golden, oracle_mod, name, model, mode):
    g = golden("link_small")
    ent, rel, ent_im, rel_im = _tables(g, name)
    pred = oracle_mod.link_predict(model, mode, ent, rel, g["qh"], g["qr"], g["qt"], ent_im=ent_im,
                                   rel_im=rel_im, **_kw(name, oracle_mod))
    ref = g[f"{name}_pred_{'head' if mode == 'head_batch' else 'tail'}"]
    assert pred.shape == ref.shape
    # float scores within 1e-4 (north_star tolerance), relative for |score| > 1
    assert np.all(np.abs(pred - ref) <= _score_tol(ref)), np.max(np.abs(pred - ref))


def _min_gap(pred, truth_idx):
    t = pred[np.arange(pred.shape[0]), truth_idx][:, None]
    gap = np.abs(pred - t)
    gap[np.arange(pred.shape[0]), truth_idx] = np.inf
    return gap.min(1)


@pytest.mark.parametrize("name,model", LINK_MODELS)
@pytest.mark.parametrize("tc", [0, 1])
def test_link_ranks_and_metrics_match_reference(golden, oracle_mod, name, model, tc):
    """Oracle ranks (Test.h restatement) on the oracle's own scores equal the reference's
    Base.so ranks on the reference's torch scores, for every query whose truth score is not
    within float noise of another candidate (near-ties are reported, not hidden)."""
    g = golden("link_small")
    ent, rel, ent_im, rel_im = _tables(g, name)
    trip = np.concatenate([np.loadtxt(f"{oracle_mod.HERE}/../tests/golden/data/small/{f}", skiprows=1,
                                      dtype=np.int64, ndmin=2) for f in ("train2id.txt", "valid2id.txt", "test2id.txt")])
    hrt = oracle_mod.sorted_hrt(trip[:, 0], trip[:, 2], trip[:, 1])
    type_off = type_ids = None
    if tc:
        type_off, type_ids = _types(oracle_mod, "small")
    counts = {}
    for mode, side in (("head_batch", "head"), ("tail_batch", "tail")):
        pred = oracle_mod.link_predict(model, mode, ent, rel, g["qh"], g["qr"], g["qt"], ent_im=ent_im,
                                       rel_im=rel_im, **_kw(name, oracle_mod))
        toff, tids = (type_off[side], type_ids[side]) if tc else (None, None)
        c = oracle_mod.test_rank(mode, pred, g["qh"], g["qr"], g["qt"], hrt, toff, tids)
        ref = g[f"{name}_tc{tc}_{side}_counts"]
        truth = g["qh"] if side == "head" else g["qt"]
        # near-tie screen: a query is decidable when every candidate is further from the
        # truth than twice the largest oracle-vs-reference score difference on that row
        err = np.abs(pred - g[f"{name}_pred_{side}"]).max(1)
        ok = _min_gap(g[f"{name}_pred_{side}"], truth) > 2 * err
        cols = [0, 1, 2, 3] if tc else [0, 1]
        assert np.array_equal(c[ok][:, cols], ref[ok][:, cols])
        assert ok.mean() > 0.97, ok.mean()
        counts[side] = np.where(ok[:, None], c, ref)
    m = oracle_mod.link_metrics(counts["head"], counts["tail"])
    grp = m["filter_tc"] if tc else m["filter"]
    got = np.array([grp[k] for k in oracle_mod.METRIC_NAMES], np.float32)
    assert np.array_equal(got, g[f"{name}_tc{tc}_metrics"])


def _types(oracle_mod, ds):
    path = f"{oracle_mod.HERE}/../tests/golden/data/{ds}/type_constrain.txt"
    with open(path) as f:
        n_rel = int(f.readline())
        heads, tails = {}, {}
        for _ in range(n_rel):
            a = list(map(int, f.readline().split()))
            heads[a[0]] = sorted(a[2:2 + a[1]])
            b = list(map(int, f.readline().split()))
            tails[b[0]] = sorted(b[2:2 + b[1]])
    out_off, out_ids = {}, {}
    for side, d in (("head", heads), ("tail", tails)):
        off = [0]
        ids = []
        for r in range(n_rel):
            ids.extend(d.get(r, []))
            off.append(len(ids))
        out_off[side] = np.array(off, np.int64)
        out_ids[side] = np.array(ids, np.int64)
    return out_off, out_ids


def test_metrics_from_reference_counts(golden, oracle_mod):
    """P14: the float accumulation of Test.h reproduced bit-exactly from the reference counts."""
    g = golden("link_small")
    for name, _ in LINK_MODELS:
        for tc in (0, 1):
            m = oracle_mod.link_metrics(g[f"{name}_tc{tc}_head_counts"], g[f"{name}_tc{tc}_tail_counts"])
            grp = m["filter_tc"] if tc else m["filter"]
            got = np.array([grp[k] for k in oracle_mod.METRIC_NAMES], np.float32)
            assert np.array_equal(got, g[f"{name}_tc{tc}_metrics"]), (name, tc, got, g[f"{name}_tc{tc}_metrics"])


def test_glibc_rand_seeds(golden, oracle_mod):
    """randReset (Random.h:11-15) seeds each work thread with the next values of the
    process-wide glibc rand() stream (default srand(1)); every recorded seed vector is a
    contiguous window of that stream."""
    stream = oracle_mod.glibc_rand(256).astype(np.uint64)
    assert stream[:3].tolist() == [1804289383, 846930886, 1681692777]
    for ds in ("small", "medium"):
        g = golden(f"sampler_{ds}")
        for key in g:
            if key.endswith("_seeds0"):
                s = g[key]
                hits = [o for o in range(len(stream) - len(s)) if np.array_equal(stream[o:o + len(s)], s)]
                assert hits, key


@pytest.mark.parametrize("ds", ["small", "medium"])
def test_sampler_bit_exact(golden, oracle_mod, ds):
    g = golden(f"sampler_{ds}")
    tr = np.loadtxt(f"{oracle_mod.HERE}/../tests/golden/data/{ds}/train2id.txt", skiprows=1, dtype=np.int64, ndmin=2)
    n_ent = int(open(f"{oracle_mod.HERE}/../tests/golden/data/{ds}/entity2id.txt").readline())
    n_rel = int(open(f"{oracle_mod.HERE}/../tests/golden/data/{ds}/relation2id.txt").readline())
    ix = oracle_mod.train_index(tr[:, 0], tr[:, 1], tr[:, 2], n_ent, n_rel)
    names = sorted({k[:-len("_cfg")] for k in g if k.endswith("_cfg")})
    for name in names:
        threads, B, neg, negrel, mode, bern = g[f"{name}_cfg"].tolist()
        seeds = g[f"{name}_seeds0"].copy()
        for step in range(3):
            bh, bt, br, by = oracle_mod.sampling(ix, seeds, B, neg, negrel, mode, bool(bern),
                                                 train_total=int(g[f"{name}_train_total"]))
            assert np.array_equal(np.stack([bh, bt, br]), g[f"{name}_step{step}"]), (name, step)
            assert np.array_equal(by, g[f"{name}_y{step}"])
        assert np.array_equal(seeds, g[f"{name}_seeds_end"])


def test_sampler_p_bit_exact(golden, oracle_mod):
    """sampling(..., p=True): the oracle's importProb table and KL-weighted corrupt_rel
    (Corrupt.h:111-147) against the reference Base.so's batches (tests/golden/make_sampler_p.py),
    including relation lists emptied by the (h, t) block (the reference returns -1)."""
    g = golden("sampler_p")
    ds = f"{oracle_mod.HERE}/../tests/golden/data/prel"
    tr = np.loadtxt(f"{ds}/train2id.txt", skiprows=1, dtype=np.int64, ndmin=2)
    n_ent, n_rel = int(open(f"{ds}/entity2id.txt").readline()), int(open(f"{ds}/relation2id.txt").readline())
    ix = oracle_mod.train_index(tr[:, 0], tr[:, 1], tr[:, 2], n_ent, n_rel)
    names = sorted({k[:-len("_cfg")] for k in g if k.endswith("_cfg")})
    empty = 0
    for name in names:
        threads, B, neg, negrel, mode, bern = g[f"{name}_cfg"].tolist()
        prob = oracle_mod.import_prob(f"{ds}/kl_prob.txt", n_rel, float(g[f"{name}_temp"]))
        assert np.array_equal(prob.ravel(), g[f"{name}_prob"]), name
        seeds = g[f"{name}_seeds0"].copy()
        for step in range(3):
            bh, bt, br, by = oracle_mod.sampling(ix, seeds, B, neg, negrel, mode, bool(bern),
                                                 train_total=int(g[f"{name}_train_total"]), prob=prob)
            assert np.array_equal(np.stack([bh, bt, br]), g[f"{name}_step{step}"]), (name, step)
            assert np.array_equal(by, g[f"{name}_y{step}"])
            empty += int((br == -1).sum())
        assert np.array_equal(seeds, g[f"{name}_seeds_end"])
    assert empty > 0  # the empty-list edge is exercised


def test_candidate_rank_rule(golden, oracle_mod):
    g = golden("repo")
    s, r = oracle_mod.candidate_rank_transe(g["ev_ent"], g["ev_rel"], g["ev_qh"], g["ev_qr"], g["ev_off"],
                                            g["ev_cids"])
    assert np.all(np.abs(s - g["ev_scores"]) <= 1e-4 * np.maximum(1, np.abs(g["ev_scores"])))
    assert np.array_equal(r, g["ev_ranks"])


def test_cosine_rank_rule(golden, oracle_mod):
    g = golden("repo")
    s, r = oracle_mod.cosine_rank(g["zs_cand"], g["zs_off"], g["zs_relvecs"], g["zs_rel"])
    assert np.allclose(s, g["zs_scores"], atol=1e-5)
    assert np.array_equal(r, g["zs_ranks"])


@pytest.mark.parametrize("tag", ["g200_eval", "g200_train", "g256_eval"])
def test_generator(golden, oracle_mod, tag):
    g = golden("repo")
    layers = [(g[f"{tag}_W{i}"], g[f"{tag}_b{i}"], g[f"{tag}_u{i}"], g[f"{tag}_v{i}"]) for i in range(3)]
    out, uv = oracle_mod.generator_forward(g[f"{tag}_noise"], g[f"{tag}_cls"], layers, g[f"{tag}_a"],
                                           g[f"{tag}_b"], train=bool(g[f"{tag}_train"]))
    assert np.allclose(out, g[f"{tag}_out"], atol=1e-4, rtol=1e-4), np.abs(out - g[f"{tag}_out"]).max()
    for i in range(3):
        assert np.allclose(uv[i][0], g[f"{tag}_u{i}_after"], atol=1e-5)
        assert np.allclose(uv[i][1], g[f"{tag}_v{i}_after"], atol=1e-5)


def test_margin_loss_and_regul(golden, oracle_mod):
    g = golden("repo")
    loss = oracle_mod.margin_loss(g["p"], g["n"], 3.0)
    assert abs(loss - g["gcn_loss"] + 0.5 * g["regul"]) < 1e-5 or abs(loss + 0.5 * g["regul"] - g["struct_loss"]) < 1e-5
    # P9 aliasing: the reported gcn_loss IS struct_loss (margin + 0.5 * regul)
    assert abs(g["gcn_loss"] - g["struct_loss"]) < 1e-7
    assert abs(oracle_mod.margin_loss(g["p"], g["n"], 3.0, adv_temperature=2.0) - g["adv_loss"]) < 1e-5


REF_TESTER_META = {
    "transe": dict(model="transe", norm_flag=True, dim=32),
    "transe_nonorm_margin": dict(model="transe", norm_flag=False, transe_margin=5.0, dim=32),
    "transe_l2": dict(model="transe_l2", norm_flag=True, dim=32),
    "distmult": dict(model="distmult", dim=32),
    "complex": dict(model="complex", dim=24),
    "rotate": dict(model="rotate", margin=6.0, epsilon=2.0, dim=16),
}


@pytest.mark.parametrize("name", sorted(REF_TESTER_META))
def test_ref_tester_predict_is_the_reference(golden, name):
    """oracle/ref_tester.py (the bench's cpu_baseline and full-size parity checker) scores
    bit-identically to the reference models' own predict() (golden link_small)."""
    import torch
    import ref_tester
    g = golden("link_small")
    ent, rel, ent_im, rel_im = _tables(g, name)
    tables = {"ent": ent, "rel": rel}
    if ent_im is not None:
        tables.update(ent_im=ent_im, rel_im=rel_im)
    predict = ref_tester.make_predict(REF_TESTER_META[name], tables)
    E = int(g["E"])
    all_e = torch.arange(E)
    for mode, key in (("head_batch", "head"), ("tail_batch", "tail")):
        ref = g[f"{name}_pred_{key}"]
        for i in range(0, len(g["qh"]), 7):
            h, r, t = (torch.tensor([int(g[k][i])]) for k in ("qh", "qr", "qt"))
            s = predict(all_e, t, r, mode) if mode == "head_batch" else predict(h, all_e, r, mode)
            np.testing.assert_array_equal(s, ref[i])


def test_ref_tester_near_ties():
    import ref_tester
    s = np.array([[1.0, 1.00005, 2.0, 0.99999], [3.0, -3.0, 2.9999, 5.0]], np.float32)
    got = ref_tester.near_ties(s, np.array([0, 2]), 1e-4)
    # row 0: tol 2e-4 -> entities 1 and 3 are near; row 1: tol 5e-4 -> entity 0 is near
    np.testing.assert_array_equal(got, [2, 1])


@pytest.mark.parametrize("name,norm,margin,adv,regul", [("transe", True, 5.0, None, 0.0),
                                                         ("transe_nonorm", False, 3.0, None, 0.5),
                                                         ("transe_adv", True, 5.0, 1.0, 0.0)])
def test_ref_trainer_loss_is_the_reference(golden, name, norm, margin, adv, regul):
    """oracle/ref_trainer.transe_ns_loss (bench --config ns cpu_baseline, float reference of the
    fused loss) == the reference strategy's loss and gradients (golden strategy.npz)."""
    import torch
    import ref_trainer
    g = golden("strategy")
    ent = torch.from_numpy(g[f"{name}.ent_embeddings.weight"]).requires_grad_(True)
    rel = torch.from_numpy(g[f"{name}.rel_embeddings.weight"]).requires_grad_(True)
    h, t, r = (torch.from_numpy(g[f"{name}_{k}"]) for k in ("h", "t", "r"))
    loss, score = ref_trainer.transe_ns_loss(ent, rel, h, t, r, int(g["B"]), margin, norm_flag=norm,
                                             adv_temperature=adv, regul_rate=regul)
    loss.backward()
    np.testing.assert_array_equal(score.detach().numpy(), g[f"{name}_score"])
    assert float(loss) == pytest.approx(float(g[f"{name}_loss"]), abs=1e-6)
    np.testing.assert_allclose(ent.grad.numpy(), g[f"{name}.grad.ent_embeddings.weight"], atol=1e-7, rtol=1e-5)
    np.testing.assert_allclose(rel.grad.numpy(), g[f"{name}.grad.rel_embeddings.weight"], atol=1e-7, rtol=1e-5)
