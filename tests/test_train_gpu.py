"""GPU parity of the training hot path: the OpenKE sampler (bit-exact vs the reference
Base.so's batches), the repo sampler (invariants), and the fused negative-sampling margin
loss + gradients (vs the reference OpenKE strategy's loss and autograd gradients)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ds", ["small", "medium"])
def test_openke_sampler_bit_exact(golden, ds):
    from mmre.data import OpenKEDataset, TrainIndex
    from mmre.sampler import OpenKESampler
    g = golden(f"sampler_{ds}")
    d = OpenKEDataset(os.path.join(GOLDEN, "data", ds))
    ix = TrainIndex(d.train[:, 0], d.train[:, 1], d.train[:, 2], d.n_ent, d.n_rel)
    names = sorted({k[:-len("_cfg")] for k in g if k.endswith("_cfg")})
    for name in names:
        threads, B, neg, negrel, mode, bern = g[f"{name}_cfg"].tolist()
        s = OpenKESampler(ix, "cuda:0", work_threads=threads, bern=bool(bern), seeds=g[f"{name}_seeds0"],
                          train_total=int(g[f"{name}_train_total"]))
        for step in range(3):
            out = s.sample(B, neg, negrel, mode)
            got = torch.stack([out["batch_h"], out["batch_t"], out["batch_r"]]).cpu().numpy()
            assert np.array_equal(got, g[f"{name}_step{step}"]), (name, step)
            assert np.array_equal(out["batch_y"].cpu().numpy(), g[f"{name}_y{step}"])
        assert np.array_equal(s.seeds, g[f"{name}_seeds_end"])
        # the device-resident states (advanced on the stream) equal Base.cpp's after 3 batches too
        assert np.array_equal(s._seeds_dev.cpu().numpy().view(np.uint64), g[f"{name}_seeds_end"])


def test_openke_sampler_p_bit_exact(golden):
    """sampling(..., p=True) on the GPU (mmre_sampler_openke_p): KL-weighted relation negatives
    bit-identical to the reference Base.so's (tests/golden/make_sampler_p.py), device seeds too."""
    from mmre.data import OpenKEDataset, TrainIndex
    from mmre.sampler import OpenKESampler
    g = golden("sampler_p")
    path = os.path.join(GOLDEN, "data", "prel")
    d = OpenKEDataset(path)
    ix = TrainIndex(d.train[:, 0], d.train[:, 1], d.train[:, 2], d.n_ent, d.n_rel)
    names = sorted({k[:-len("_cfg")] for k in g if k.endswith("_cfg")})
    for name in names:
        threads, B, neg, negrel, mode, bern = g[f"{name}_cfg"].tolist()
        s = OpenKESampler(ix, "cuda:0", work_threads=threads, bern=bool(bern), seeds=g[f"{name}_seeds0"],
                          train_total=int(g[f"{name}_train_total"]))
        prob = s.import_prob(os.path.join(path, "kl_prob.txt"), float(g[f"{name}_temp"]))
        assert np.array_equal(prob.ravel(), g[f"{name}_prob"])
        for step in range(3):
            out = s.sample(B, neg, negrel, mode, p=True)
            got = torch.stack([out["batch_h"], out["batch_t"], out["batch_r"]]).cpu().numpy()
            assert np.array_equal(got, g[f"{name}_step{step}"]), (name, step)
            assert np.array_equal(out["batch_y"].cpu().numpy(), g[f"{name}_y{step}"])
        assert np.array_equal(s._seeds_dev.cpu().numpy().view(np.uint64), g[f"{name}_seeds_end"])


def test_openke_sampler_full_size_properties():
    """FB15K237-sized synthetic train set (272,115 triples), B = 2,721, k = 25, 8 threads:
    every entity negative avoids the filter set of its positive (Corrupt.h:7-81)."""
    from mmre.data import TrainIndex
    from mmre.sampler import OpenKESampler
    rng = np.random.default_rng(3)
    E, R, n = 14541, 237, 272115
    h, t, r = rng.integers(0, E, n), rng.integers(0, E, n), rng.integers(0, R, n)
    ix = TrainIndex(h, t, r, E, R)
    s = OpenKESampler(ix, "cuda:0", work_threads=8, bern=True)
    out = s.sample(2721, 25, 0, 0)
    bh, bt, br = (out[k].cpu().numpy() for k in ("batch_h", "batch_t", "batch_r"))
    known = set(map(tuple, ix.train_list.tolist()))
    B = 2721
    for j in range(1, 26):
        sl = slice(j * B, (j + 1) * B)
        assert np.all(br[sl] == br[:B])
        for a, b2, c in zip(bh[sl][:300], br[sl][:300], bt[sl][:300]):
            assert (a, b2, c) not in known
    assert np.all((bh >= 0) & (bh < E) & (bt >= 0) & (bt < E))


def test_repo_sampler_invariants():
    from mmre.sampler import RepoSampler
    rng = np.random.default_rng(4)
    G, R, N, B, k = 800, 23, 60, 48, 10
    wh, wr, wt = rng.integers(0, G, 3000), rng.integers(0, R, 3000), rng.integers(0, G, 3000)
    l2g = rng.permutation(G)[:N]
    eh, et = rng.integers(0, N - 1, B), rng.integers(0, N - 1, B)
    er = rng.integers(0, R, B)
    wh = np.concatenate([wh, l2g[eh]]); wt = np.concatenate([wt, l2g[et]]); wr = np.concatenate([wr, er])
    s = RepoSampler([wh, wr, wt], R, "cuda:0", seed=1)
    dev = torch.device("cuda:0")
    ei, et2 = s.sample(torch.from_numpy(np.stack([eh, et])).to(dev), torch.from_numpy(er).to(dev), k, N - 1,
                       torch.from_numpy(l2g).to(dev))
    ei = ei.cpu().numpy(); et2 = et2.cpu().numpy()
    known_h = {}
    for a, b2, c in zip(wh, wr, wt):
        known_h.setdefault((c, b2), set()).add(a)
    known_t = {}
    for a, b2, c in zip(wh, wr, wt):
        known_t.setdefault((a, b2), set()).add(c)
    assert np.array_equal(ei[0, :B], eh) and np.array_equal(ei[1, :B], et) and np.array_equal(et2[:B], er)
    for j in range(1, k + 1):
        for b in range(B):
            row = j * B + b
            h2, t2 = ei[0, row], ei[1, row]
            assert 0 <= h2 < N - 1 and 0 <= t2 < N - 1
            assert et2[row] == er[b]
            if h2 != eh[b]:
                assert t2 == et[b] and l2g[h2] not in known_h.get((l2g[et[b]], er[b]), set())
            elif t2 != et[b]:
                assert l2g[t2] not in known_t.get((l2g[eh[b]], er[b]), set())


STRAT = [("transe", "transe", dict(norm=True), 5.0, None, 0.0),
         ("transe_nonorm", "transe", dict(norm=False), 3.0, None, 0.5),
         ("transe_adv", "transe", dict(norm=True), 5.0, 1.0, 0.0),
         ("distmult", "distmult", {}, 5.0, None, 0.25),
         ("complex", "complex", {}, 4.0, None, 0.1),
         ("rotate", "rotate", {}, 6.0, 2.0, 0.0)]


@pytest.mark.parametrize("name,model,kw,margin,adv,regul", STRAT)
def test_fused_ns_loss_and_grads(golden, name, model, kw, margin, adv, regul):
    from mmre.link import rotate_phase_denom
    from mmre.ns import NSSpec, fused_ns_loss
    g = golden("strategy")
    dev = torch.device("cuda:0")
    B, k = int(g["B"]), int(g["k"])
    P = lambda key: torch.from_numpy(g[f"{name}.{key}"]).to(dev).requires_grad_(True)
    if model == "complex":
        ent, ent_im, rel, rel_im = (P(x) for x in ("ent_re_embeddings.weight", "ent_im_embeddings.weight",
                                                   "rel_re_embeddings.weight", "rel_im_embeddings.weight"))
        dim = ent.shape[1]
    else:
        ent, rel = P("ent_embeddings.weight"), P("rel_embeddings.weight")
        ent_im = rel_im = None
        dim = rel.shape[1]
    spec = NSSpec(model, dim, norm_flag=kw.get("norm", False),
                  model_margin=6.0 if model == "rotate" else None,
                  phase_denom=rotate_phase_denom(6.0, 2.0, dim) if model == "rotate" else 0.0)
    h, t, r = (torch.from_numpy(g[f"{name}_{x}"]).to(dev) for x in ("h", "t", "r"))
    loss, score = fused_ns_loss(spec, ent, rel, h, t, r, B, k, margin, adv, regul, ent_im=ent_im, rel_im=rel_im)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - float(g[f"{name}_loss"])) <= 1e-4 * max(1.0, abs(float(g[f"{name}_loss"])))
    ref_s = g[f"{name}_score"]
    assert np.all(np.abs(score.cpu().numpy() - ref_s) <= 1e-4 * np.maximum(1, np.abs(ref_s)))
    pairs = [("ent_embeddings.weight", ent), ("rel_embeddings.weight", rel)]
    if model == "complex":
        pairs = [("ent_re_embeddings.weight", ent), ("ent_im_embeddings.weight", ent_im),
                 ("rel_re_embeddings.weight", rel), ("rel_im_embeddings.weight", rel_im)]
    for key, p in pairs:
        ref = g[f"{name}.grad.{key}"]
        got = p.grad.cpu().numpy()
        scale = max(np.abs(ref).max(), 1e-12)
        assert np.abs(got - ref).max() <= 1e-4 * scale + 1e-7, (key, np.abs(got - ref).max(), scale)


def test_repo_negative_sampling_loss(golden):
    """module/NegativeSampling.py forward loss assembly: TransE L1 over local GCN rows with
    per-positive relation rows; margin 3, regul 0.5 (P9 aliasing: gcn_loss is struct_loss)."""
    from mmre.ns import NSSpec, fused_ns_loss
    g = golden("repo")
    dev = torch.device("cuda:0")
    x = torch.from_numpy(g["x"]).to(dev)
    rel = torch.from_numpy(g["rel"]).to(dev)
    B = rel.shape[0]
    k = g["eh"].shape[0] // B - 1
    h = torch.from_numpy(g["eh"].astype(np.int64)).to(dev)
    t = torch.from_numpy(g["et"].astype(np.int64)).to(dev)
    r = torch.arange(B, device=dev).repeat(1 + k)
    loss, score = fused_ns_loss(NSSpec("transe", 48), x, rel, h, t, r, B, k, 3.0, None, 0.5)
    torch.cuda.synchronize()
    assert abs(loss.item() - float(g["struct_loss"])) < 1e-4 * max(1, abs(float(g["struct_loss"])))
    assert np.allclose(score.cpu().numpy(), g["score"], rtol=1e-4, atol=1e-4)


def test_hip_sgd_step_matches_torch():
    """mmre.optim.SGD: the plain step is one HIP launch (mmre_sgd_step) over up to 8 tensors
    per launch, float4 streams with a scalar tail; p - lr g as one fma with lr in float32,
    bit-identical to torch's default (foreach) SGD step on this ROCm build, which is that same
    fma (scripts/probes/sgd_rounding.py: 0 differences vs the fma at lr 1 / 0.1 / 0.0123 / 1e-4,
    ~20 % vs a rounded multiply then add); momentum / weight decay run torch's own step."""
    from mmre.optim import SGD
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(14208, 200), (235, 200), (7,), (1, 5), (1031,)] + [(33, 3)] * 6   # 11 tensors: 2 launches
    ref = [torch.randn(s, generator=g).to(dev) for s in shapes]
    mine = [r.clone() for r in ref]
    grads = [torch.randn(s, generator=g).to(dev) for s in shapes]
    for ps in (ref, mine):
        for p, gr in zip(ps, grads):
            p.grad = gr.clone()
    torch.optim.SGD(ref, lr=0.37).step()
    before = SGD.fallback_steps
    SGD(mine, lr=0.37).step()
    assert SGD.fallback_steps == before          # the HIP step ran
    torch.cuda.synchronize()
    for a, b in zip(ref, mine):
        assert torch.equal(a, b), (a != b).sum().item()
    # options the kernel does not cover: torch's own step, bit for bit
    ref2 = [r.clone() for r in ref]
    mine2 = [r.clone() for r in ref]
    for ps in (ref2, mine2):
        for p, gr in zip(ps, grads):
            p.grad = gr.clone()
    torch.optim.SGD(ref2, lr=0.1, momentum=0.9, weight_decay=0.01).step()
    SGD(mine2, lr=0.1, momentum=0.9, weight_decay=0.01).step()
    for a, b in zip(ref2, mine2):
        assert torch.equal(a, b)
