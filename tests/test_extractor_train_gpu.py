"""GPU tests of the Extractor's training mode and its pretraining step (pretrain_Extractor,
module/zsl_module.py:289-348; mmre/extractor_train.py + csrc/extractor_train.hip).

Oracle: oracle/zsl_extractor.py's train_encode_ref / pretrain_step_ref, a literal torch
restatement of the reference's training-mode forward (per-slot gcn_w then the slot sum, every
nn.Dropout replaced by an injected 0/1 mask), margin loss, backward and torch.optim.Adam, run in
float64. Parity unpinned by reference fixtures (the reference ships none and running its Python
is denied).

Bars: with the same injected masks, loss within 1e-5 relative, every gradient within 1e-4 of its
tensor's largest entry, every updated weight within 1e-6 wherever the gradient is not within
rounding of zero (Adam's first step is lr * g / |g|, a sign); p = 0 equals the eval-mode fused
encode; the counter-hash masks keep 80 % at p 0.2, are reproducible per (seed, offset) and fresh
after advance(); a hipGraph replay equals the eager step; pretraining lowers the loss.
"""
import random

import numpy as np
import pytest
import torch

from zsl_synth import embeddings, init_extractor, make_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _setup(d=200, seed=0):
    from module.zsl_module import Extractor, ZSLGraph
    g = make_graph(seed=seed)
    ent, rel = embeddings(g, d)
    graph = ZSLGraph(g["rel2id"], g["ent2id"], g["train_tasks"], g["test_tasks"], ent, rel, max_neighbor=50)
    ex = Extractor(d, graph.num_symbols, graph.symbol2vec)
    init_extractor(ex)
    return g, graph, ex


def _generator(g, graph, batch_size=16, few=4, sub_epoch=3, seed=0):
    """Extractor_generate over the synthetic graph; candidate pools hold entities with
    neighbours only (a degree-0 entity divides by zero in the reference's neighbour encoder)."""
    from mmre.extractor_train import extractor_generate
    rng = np.random.default_rng(seed)
    live = [e for e in g["ents"] if graph.e1_degrees[g["ent2id"][e]] > 0]
    rel2cand = {r: [live[i] for i in rng.choice(len(live), 60, replace=False)] for r in g["rels"]}
    e1rel_e2 = {}
    for tasks in (g["train_tasks"], g["test_tasks"]):
        for _, tri in tasks.items():
            for h, r, t in tri:
                e1rel_e2.setdefault(h + r, []).append(t)
    tasks = {k: list(v) for k, v in g["train_tasks"].items()}
    return extractor_generate(tasks, rel2cand, e1rel_e2, g["ent2id"], batch_size, few, sub_epoch,
                              random.Random(seed))


def _step(graph, ex, **kw):
    from mmre.extractor_train import PretrainStep
    return PretrainStep(ex, torch.as_tensor(graph.ent_sym), torch.as_tensor(graph.connections),
                        torch.as_tensor(graph.e1_degrees, dtype=torch.float32), **kw)


def _dev(batch):
    return {k: torch.as_tensor(v, device=DEV) for k, v in batch.items()}


@pytest.mark.parametrize("d", [200, 100])
def test_pretrain_step_matches_oracle_with_injected_masks(d):
    import zsl_extractor as ox
    g, graph, ex = _setup(d)
    ref = ox.ExtractorRef(d, graph.num_symbols, graph.symbol2vec)
    ref.load_state_dict({k: v for k, v in ex.state_dict().items()}, strict=True)
    ref = ref.double()
    ex = ex.to(DEV).train()
    lr, margin = 1e-3, 5.0
    step = _step(graph, ex, lr=lr, margin=margin, seed=1)
    step.keep_grads = True
    b = next(_generator(g, graph))
    S, Q, F_ = len(b["s_h"]), len(b["q_h"]), len(b["f_h"])
    heads = np.concatenate([b["s_h"], b["q_h"], b["s_h"], b["f_h"]])
    tails = np.concatenate([b["s_t"], b["q_t"], b["s_t"], b["f_t"]])
    N, M = len(heads), graph.connections.shape[1]
    rng = np.random.default_rng(5)
    masks = [(rng.random(s) >= 0.2).astype(np.uint8) for s in ((N, M, d), (N, M, d), (N, 2, d), (N, d))]
    bd = _dev(b)
    loss = step.step(bd["s_h"], bd["s_t"], bd["q_h"], bd["q_t"], bd["f_h"], bd["f_t"],
                     masks=[torch.from_numpy(m) for m in masks])
    pairs = torch.from_numpy(np.stack([graph.ent_sym[heads], graph.ent_sym[tails]], 1))
    meta = ox.get_meta(graph.connections, graph.e1_degrees, heads, tails)
    meta = (meta[0], meta[1].double(), meta[2], meta[3].double())
    r_loss, r_grads, r_new = ox.pretrain_step_ref(ref, pairs, meta, (S, Q, F_), masks, margin, lr)
    assert float(r_loss) > 0.1                                     # the hinge is active
    assert abs(float(loss) - float(r_loss)) <= 1e-5 * abs(float(r_loss))
    names = [n for n, q in ex.named_parameters() if q.requires_grad]
    for n, gg in zip(names, step.grads):
        rg = r_grads[n]
        if rg is None:
            assert gg is None or float(gg.abs().max()) == 0.0, n
            continue
        err = (gg.double().cpu() - rg).abs().max().item()
        assert err <= 1e-4 * max(rg.abs().max().item(), 1e-12), (n, err, rg.abs().max().item())
    new = dict(ex.named_parameters())
    for n in names:
        if r_grads[n] is None:
            continue
        rg = r_grads[n]
        live = rg.abs() > 1e-3 * rg.abs().max()
        diff = (new[n].detach().double().cpu() - r_new[n]).abs()
        assert diff[live].max().item() <= 1e-6, (n, diff[live].max().item())
        assert diff.max().item() <= 2.0 * lr + 1e-6


def test_p0_train_forward_equals_eval_encode():
    from mmre.extractor_train import DropoutRNG, train_forward
    g, graph, ex = _setup(200)
    ex = ex.to(DEV)
    idx = np.arange(64)
    heads = np.array([graph.ent2id[e] for e in g["ents"][:64]])
    tails = np.array([graph.ent2id[e] for e in g["ents"][64:128]])
    pairs = torch.as_tensor(np.stack([graph.ent_sym[heads], graph.ent_sym[tails]], 1), device=DEV)
    meta = graph.get_meta(heads, tails, device=DEV)
    ex.eval()
    ref_g, _ = ex.encode_pairs(pairs, meta)
    ex.train()
    with torch.no_grad():
        gt = train_forward(ex, pairs, meta, p=0.0, rng=DropoutRNG(0, DEV))
    ok = torch.isfinite(ref_g).all(1)
    assert int(ok.sum()) >= len(idx) - 2
    assert torch.allclose(gt[ok], ref_g[ok], atol=2e-5, rtol=0)


def test_dropout_masks_counter_hash():
    from mmre._lib import call, ptr, stream_ptr
    from mmre.extractor_train import DropoutRNG
    n = 1 << 21
    x = torch.ones(n, device=DEV)
    rng = DropoutRNG(123, DEV)

    def draw(stream_id=0):
        y = torch.empty_like(x)
        m = torch.empty(n, dtype=torch.uint8, device=DEV)
        call("mmre_dropout", ptr(x), ptr(y), ptr(m), n, 0.2, ptr(rng.state), stream_id, stream_ptr(DEV))
        return y, m

    y0, m0 = draw()
    keep = m0.float().mean().item()
    assert abs(keep - 0.8) < 0.002
    assert torch.equal(y0, m0.float() * 1.25)                      # kept values x / (1 - p) = 1.25 exactly
    y1, m1 = draw()
    assert torch.equal(m0, m1)                                     # same (seed, offset, stream): same mask
    _, m2 = draw(stream_id=3)
    rng.advance()
    _, m3 = draw()
    for other in (m2, m3):                                         # fresh masks: agreement ~ 0.8^2 + 0.2^2
        agree = (other == m0).float().mean().item()
        assert abs(agree - 0.68) < 0.003
    # neighbour / entity masks of the gather kernel keep 80 % as well
    g, graph, ex = _setup(200)
    from mmre.extractor_train import train_inputs
    heads = np.arange(128) % graph.num_ents
    pairs = torch.as_tensor(np.stack([graph.ent_sym[heads]] * 2, 1), device=DEV)
    meta = graph.get_meta(heads, heads, device=DEV)
    emb = torch.as_tensor(graph.symbol2vec, dtype=torch.float32, device=DEV)
    _, _, e1, e2 = train_inputs(emb, pairs, meta, 0.2, DropoutRNG(7, DEV))
    src = emb[pairs[:, 0]]
    nz = src != 0
    kept = ((e1 != 0) & nz).float().sum() / nz.float().sum()
    assert abs(kept.item() - 0.8) < 0.01
    assert torch.equal(e1[e1 != 0], src[e1 != 0] * 1.25)
    assert not torch.equal(e1 != 0, e2 != 0)                       # the two entity rows draw their own masks


def test_replay_equals_eager_and_pretraining_learns():
    import copy
    g, graph, ex = _setup(200)
    ex = ex.to(DEV).train()
    ex2 = copy.deepcopy(ex)
    a = _step(graph, ex, lr=1e-3, seed=9)
    b = _step(graph, ex2, lr=1e-3, seed=9)
    batch = _dev(next(_generator(g, graph, batch_size=32, few=6, sub_epoch=4)))
    keys = ("s_h", "s_t", "q_h", "q_t", "f_h", "f_t")
    eager = [float(a.step(*(batch[k] for k in keys))) for _ in range(4)]
    graphed = [float(b.replay(batch)) for _ in range(4)]
    assert len(set(eager)) == 4                                    # fresh masks (and weights) every step
    np.testing.assert_allclose(graphed, eager, rtol=1e-5)
    for p1, p2 in zip(ex.parameters(), ex2.parameters()):
        assert torch.allclose(p1, p2, atol=1e-6)
    # pretraining on the generator's batches lowers the margin loss
    gen = _generator(g, graph, batch_size=32, few=6, sub_epoch=4, seed=1)
    losses = [float(b.replay(_dev(next(gen)))) for _ in range(300)]
    assert np.all(np.isfinite(losses))
    assert np.mean(losses[-50:]) < 0.9 * np.mean(losses[:50])


def test_extractor_forward_training_mode_is_differentiable():
    g, graph, ex = _setup(200)
    ex = ex.to(DEV).train()
    heads = np.array([graph.ent2id[e] for e in g["ents"][:40]])
    tails = np.array([graph.ent2id[e] for e in g["ents"][40:80]])
    q = torch.as_tensor(np.stack([graph.ent_sym[heads], graph.ent_sym[tails]], 1), device=DEV)
    meta = graph.get_meta(heads, tails, device=DEV)
    qg, scores = ex(q[8:], q[:8], tuple(m[8:] for m in meta), tuple(m[:8] for m in meta))
    assert qg.shape == (32, 200) and scores.shape == (32,)
    scores.sum().backward()
    assert ex.fc1.weight.grad is not None and float(ex.fc1.weight.grad.abs().sum()) > 0
    qg2, _ = ex(q[8:], q[:8], tuple(m[8:] for m in meta), tuple(m[:8] for m in meta))
    assert not torch.equal(qg, qg2)                                # each call draws its own masks
