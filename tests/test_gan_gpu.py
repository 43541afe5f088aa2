"""GPU parity of the zero-shot GAN step (mmre.gan.ZSLGANStep: HIP Extractor vectors, HIP
generator forward/backward, torch-ROCm Discriminator + gradient penalty, hipGraph replay)
against the float64 restatement of ZSLmodule.train's D and G steps (oracle/zsl_gan.py;
zsl_module.py:419-600, module/utils.py:692-707). Losses and gradients within 1e-4 relative;
the hipGraph replay reproduces the eager step."""
import numpy as np
import pytest
import torch

from zsl_synth import embeddings, init_extractor, make_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _setup(seed=0, n_labels=6, rows_per_rel=16):
    import zsl_extractor as ox
    from mmre.extractor import ZSLRanker
    from mmre.gan import ZSLGANStep
    from mmre.generator import RelationGenerator
    from module.zsl_module import Discriminator, Extractor, ZSLGraph
    torch.manual_seed(seed)
    g = make_graph(seed=seed, n_ent=300)
    ent, rel = embeddings(g, 200, seed=seed + 1)
    G = ZSLGraph(g["rel2id"], g["ent2id"], g["train_tasks"], g["test_tasks"], ent, rel, max_neighbor=50)
    ref = ox.ExtractorRef(200, G.num_symbols, G.symbol2vec)
    init_extractor(ref, seed=seed + 2)
    ex = Extractor(200, G.num_symbols, G.symbol2vec)
    ex.load_state_dict(ref.state_dict())
    ex = ex.to(DEV).eval()
    ranker = ZSLRanker(ex, G.ent_sym, G.connections, G.e1_degrees, device=DEV)
    gen = RelationGenerator(384, 15, 200).to(DEV)
    disc = Discriminator().to(DEV)
    with torch.no_grad():
        for p in list(gen.parameters()) + list(disc.parameters()):
            if p.dim() == 1:
                p.add_(0.05 * torch.randn_like(p))
    n_rel_ids = len(g["rel2id"])
    cls_table = torch.randn(n_rel_ids, 384, device=DEV)
    centroids = torch.randn(n_labels, 200, device=DEV)
    step = ZSLGANStep(gen, disc, cls_table, centroids, ranker, pretrain_margin=5.0, gan_batch_rela=2)
    rng = np.random.default_rng(seed)
    n = 2 * rows_per_rel
    labels = np.repeat(rng.choice(n_labels, 2, replace=False), rows_per_rel)
    batch = dict(rel=torch.as_tensor(rng.integers(0, n_rel_ids, n)), q_head=torch.as_tensor(rng.integers(0, 300, n)),
                 q_tail=torch.as_tensor(rng.integers(0, 300, n)), f_head=torch.as_tensor(rng.integers(0, 300, n)),
                 f_tail=torch.as_tensor(rng.integers(0, 300, n)), labels=torch.as_tensor(labels))
    batch = {k: v.to(DEV) for k, v in batch.items()}
    return step, batch


def _ref_of(step):
    import zsl_gan as og
    d = {k: v.detach().double().cpu().clone() for k, v in step.D.state_dict().items()}
    for k in d:
        if not (k.endswith("weight_u") or k.endswith("weight_v")):
            d[k].requires_grad_(True)
    G = step.G
    layers = [(L.weight_orig.detach().double().cpu().clone().requires_grad_(), L.bias.detach().double().cpu()
               .clone().requires_grad_(), L.weight_u.double().cpu().clone(), L.weight_v.double().cpu().clone())
              for L in (G.generate_fc_layer, G.des_rel_map_layer1, G.des_rel_map_layer2)]
    a = G.ln_a.detach().double().cpu().clone().requires_grad_()
    b = G.ln_b.detach().double().cpu().clone().requires_grad_()
    return og.GANRef(d, (layers, a, b), step.centroids.double().cpu(), margin=step.margin,
                     gan_batch_rela=step.gan_batch_rela)


def _close(a, b, what):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    scale = b.abs().max().item()
    assert (a - b).abs().max().item() <= 1e-4 * scale + 1e-6, (what, (a - b).abs().max().item(), scale)


def test_d_and_g_step_match_reference():
    step, batch = _setup()
    ref = _ref_of(step)
    n = batch["q_head"].shape[0]
    noise = torch.randn(n, 15, device=DEV)
    alpha = torch.rand(n, 1, device=DEV)
    real = step.extractor_vecs(batch["q_head"], batch["q_tail"]).double().cpu()
    neg = step.extractor_vecs(batch["f_head"], batch["f_tail"]).double().cpu()
    cls_rows = step.cls_table.index_select(0, batch["rel"]).double().cpu()
    labels = batch["labels"].cpu()
    step.keep_grads = True
    got = step.d_step(batch["rel"], batch["q_head"], batch["q_tail"], batch["f_head"], batch["f_tail"],
                      batch["labels"], noise, alpha)
    want, want_g = ref.d_step(cls_rows, real, neg, labels, noise.double().cpu(), alpha.double().cpu())
    _close(got, want, "D losses")
    for i, (x, y) in enumerate(zip(step.grads_d, want_g)):
        _close(x, y, f"D grad {i}")
    for k, v in step.D.state_dict().items():  # u, v after the four power iterations
        if k.endswith("weight_u") or k.endswith("weight_v"):
            _close(v, ref.D[k], k)
    noise2 = torch.randn(n, 15, device=DEV)
    got = step.g_step(batch["rel"], batch["q_head"], batch["q_tail"], batch["f_head"], batch["f_tail"],
                      batch["labels"], noise2)
    want, want_g = ref.g_step(cls_rows, real, neg, labels, noise2.double().cpu())
    _close(got, want, "G losses")
    for i, (x, y) in enumerate(zip(step.grads_g, want_g)):
        _close(x, y, f"G grad {i}")


def test_graph_replay_matches_eager():
    """Two identical models: one steps eagerly, one through the captured hipGraphs, with the same
    fixed noise / alpha (draw=False): losses and parameters agree after every step."""
    s1, batch = _setup(seed=3)
    s2, _ = _setup(seed=3)
    n = batch["q_head"].shape[0]
    gen = torch.Generator(device=DEV).manual_seed(7)
    for it in range(3):
        noise = torch.randn(n, 15, device=DEV, generator=gen)
        alpha = torch.rand(n, 1, device=DEV, generator=gen)
        a = s1.d_step(batch["rel"], batch["q_head"], batch["q_tail"], batch["f_head"], batch["f_tail"],
                      batch["labels"], noise, alpha)
        b = s2.replay("d", dict(batch, noise=noise, alpha=alpha), draw=False).clone()
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (it, a, b)
        a = s1.g_step(batch["rel"], batch["q_head"], batch["q_tail"], batch["f_head"], batch["f_tail"],
                      batch["labels"], noise)
        b = s2.replay("g", dict(batch, noise=noise), draw=False).clone()
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (it, a, b)
    torch.cuda.synchronize()
    for p, q in zip(list(s1.G.parameters()) + list(s1.D.parameters()), list(s2.G.parameters()) + list(s2.D.parameters())):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-6)
    # drawing mode runs and moves the parameters
    before = [p.detach().clone() for p in s2.G.parameters()]
    for _ in range(2):
        s2.replay("d", batch)
        s2.replay("g", batch)
    torch.cuda.synchronize()
    assert any(not torch.equal(x, p) for x, p in zip(before, s2.G.parameters()))
