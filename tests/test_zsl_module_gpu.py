"""GPU tests of the repo-level drop-in surface end to end:
UnifiedModel.generate / forward_relation_emb / generate_rel_embed('seen') against the oracle
chain (oracle/m3ae_text.py CLS over the full padded rows -> oracle.generator_forward /
spectral-norm + Linear in float64), ZSLmodule.eval against the oracle's per-query loop
(oracle/zsl_extractor.zsl_eval_ranks, sklearn cosine + argsort), ZSLmodule.train's GAN loop
and main.main's training / save / ZSL cadence on a synthetic zero-shot dataset directory.
Parity of these pieces is unpinned by reference fixtures (none exist; oracle headers)."""
import json
import os

import numpy as np
import pytest
import torch

from zsl_synth import candidates, embeddings, make_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _write_dataset(root, g, seed=0):
    rng = np.random.default_rng(seed)
    os.makedirs(root, exist_ok=True)
    ents = g["ents"]
    n_rel = max(g["rel2id"].values()) + 1
    words = ["film", "person", "located", "in", "the", "of", "award", "nominee", "team", "sport", "music", "genre"]
    desc = [" ".join(rng.choice(words, 3 + int(rng.integers(0, 12)))) + "." for _ in range(n_rel)]
    rel2cand = {r: [ents[i] for i in rng.choice(len(ents), 60, replace=False)] for r in g["rels"]}
    e1rel_e2 = {}
    for tasks in (g["train_tasks"], g["test_tasks"]):
        for rel, tri in tasks.items():
            for h, r, t in tri:
                e1rel_e2.setdefault(h + r, []).append(t)
    files = {"entity2ids_zsl.json": g["ent2id"], "relation2ids.json": g["rel2id"],
             "train_tasks_zsl.json": g["train_tasks"], "test_tasks_zsl.json": g["test_tasks"],
             "rel2candidates_all.json": rel2cand, "e1rel_e2_all.json": e1rel_e2,
             "test_candidates.json": candidates(g, n_cand=40, seed=seed + 1)}
    for name, obj in files.items():
        with open(os.path.join(root, name), "w") as f:
            json.dump(obj, f)
    with open(os.path.join(root, "rel_description_zsl"), "w") as f:
        f.write("\n".join(desc) + "\n")
    os.makedirs(os.path.join(root, "test"), exist_ok=True)
    with open(os.path.join(root, "test", "test_candidates.json"), "w") as f:
        json.dump(files["test_candidates.json"], f)


def _args(tmp, **kw):
    from args import read_options
    a = read_options([])
    a.model_type, a.save_path = "tiny", os.path.join(tmp, "Embed_used")
    a.train_times, a.loss_every, a.G_batch_size = 3, 1, 64
    a.pretrain_times, a.pretrain_loss_every, a.pretrain_batch_size, a.pretrain_subepoch = 12, 4, 16, 3
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _setup(tmp_path, seed=0):
    from module.data import ZSDataset
    from module.model import UnifiedModel
    g = make_graph(seed=seed)
    root = str(tmp_path / "FB-synth")
    _write_dataset(root, g, seed)
    args = _args(str(tmp_path))
    ds = ZSDataset(root, max_len=64)
    torch.manual_seed(seed)
    um = UnifiedModel(args, 200, ds, ds.num_relations, args.noise_dim)
    with torch.no_grad():  # non-trivial layer-norm affine so its parameters matter
        um.layer_norm.a_2.uniform_(0.5, 1.5)
        um.layer_norm.b_2.uniform_(-0.2, 0.2)
    return g, root, args, ds, um.to(DEV)


def _oracle_cls(um, tok, msk):
    import m3ae_text as om
    sd = {k: v.detach().cpu() for k, v in um.M3AEmodel.state_dict().items()}
    cls, _ = om.forward_representation_text(sd, tok.cpu(), msk.cpu(), um.M3AEmodel.num_heads)
    return cls[:, 0].double()


def _layers(um):
    return [(L.weight_orig.detach().cpu().numpy(), L.bias.detach().cpu().numpy(), L.weight_u.cpu().numpy(),
             L.weight_v.cpu().numpy()) for L in (um.generate_fc_layer, um.des_rel_map_layer1, um.des_rel_map_layer2)]


def _close(got, ref, tol=1e-4):
    det = lambda x: x.detach().cpu() if torch.is_tensor(x) else x
    got, ref = np.asarray(det(got), np.float64), np.asarray(det(ref), np.float64)
    err = np.abs(got - ref).max()
    assert err <= tol * max(1.0, np.abs(ref).max()), err


def test_generate_matches_oracle_chain(tmp_path):
    import oracle
    g, root, args, ds, um = _setup(tmp_path)
    um.eval()
    b = ds.generate_batch([], torch.tensor([3, 3, 3, 7, 7, 0]))
    noise = 0.1 * torch.randn(6, 15, device=DEV)
    out = um.generate(b["rel_des"].to(DEV), b["rel_des_padding_mask"].to(DEV), noise)
    cls = _oracle_cls(um, b["rel_des"], b["rel_des_padding_mask"])
    ref, _ = oracle.generator_forward(noise.cpu().numpy(), cls.numpy(), _layers(um), um.layer_norm.a_2.detach().cpu(),
                                      um.layer_norm.b_2.detach().cpu())
    _close(out.cpu(), ref)


@pytest.mark.parametrize("train_mode", [False, True])
def test_generate_rel_embed_seen_matches_oracle(tmp_path, train_mode):
    """generate_rel_embed('seen') (utils.py:529-546) = forward_relation_emb over every relation
    description: CLS -> SN des_rel_map_layer1 -> SN des_rel_map_layer2 (one power iteration per
    layer in training mode, spectral_norm.py:74-85) -- the LayerNormalization output discarded
    (model.py:609)."""
    import oracle
    from module.loss import MarginLoss
    from module.NegativeSampling import NegativeSampling
    from module.utils import generate_rel_embed
    g, root, args, ds, um = _setup(tmp_path)
    um.train(train_mode)
    layers = _layers(um)[1:]
    strat = NegativeSampling(args, ds.triples, um, MarginLoss(margin=3.0))
    got = generate_rel_embed(ds, strat, None, DEV, "seen")
    x = _oracle_cls(um, ds.rel_tokens, ds.rel_mask).numpy()
    uv = []
    for (w, bias, u, v) in layers:
        wn, u2, v2 = oracle._sn_weight(w, u, v, train_mode)
        uv.append((u2, v2))
        x = x @ wn.T + bias
    assert got.shape == (ds.num_relations, 200)
    _close(got, x)
    if train_mode:  # the power iteration updated u, v in place, as the reference's hook does
        for L, (u2, v2) in zip((um.des_rel_map_layer1, um.des_rel_map_layer2), uv):
            _close(L.weight_u.cpu(), u2, 1e-5)
            _close(L.weight_v.cpu(), v2, 1e-5)


def test_zsl_module_eval_end_to_end(tmp_path):
    """ZSLmodule(args, data_path, r2id, e2id, device, dataset).update_embed + eval(generate_model)
    == the reference loop's ranks (oracle) for every query outside near ties."""
    import oracle
    import zsl_extractor as ox
    from module.zsl_module import ZSLmodule
    g, root, args, ds, um = _setup(tmp_path, seed=4)
    zsl = ZSLmodule(args, root, ds.r2id, ds.e2id, DEV, ds)
    ent, rel = embeddings(g, 200, seed=5)
    zsl.update_embed(ent, rel)
    with torch.no_grad():
        for n, p in zsl.Extractor.named_parameters():
            if n.endswith("bias") and not n.startswith("symbol_emb"):
                p.copy_(0.05 * torch.randn_like(p))
    hits10, hits5, mrr = zsl.eval(um, mode="test", meta=True)
    # oracle chain: CLS (full padded rows) -> float64 generator -> per-query Extractor + sklearn cosine
    cands = json.load(open(os.path.join(root, "test_candidates.json")))
    ref_ex = ox.ExtractorRef(200, zsl.num_symbols, zsl.symbol2vec)
    ref_ex.load_state_dict({k: v.cpu() for k, v in zsl.Extractor.state_dict().items()}, strict=True)
    rel_vecs = {}
    for r in cands:
        rid = ds.r2id[r]
        cls = _oracle_cls(um, ds.rel_tokens[rid:rid + 1], ds.rel_mask[rid:rid + 1]).numpy()
        out, _ = oracle.generator_forward(zsl.test_noises.cpu().numpy(), np.repeat(cls, 20, 0), _layers(um),
                                          um.layer_norm.a_2.detach().cpu(), um.layer_norm.b_2.detach().cpu())
        rel_vecs[r] = out.astype(np.float32)
    o_ranks, o_scores = ox.zsl_eval_ranks(ref_ex, zsl.symbol2id, ds.e2id, zsl.connections,
                                          dict(enumerate(zsl.e1_degrees)), rel_vecs, cands)
    (g_ranks, _), _ = __import__("module.zsl_module", fromlist=["ZSLEvaluator"]).ZSLEvaluator(
        zsl.Extractor, zsl.graph, device=DEV).rank(dict(zip(cands, zsl.relation_vectors(um, list(cands)))), cands,
                                                     return_scores=True)
    g_ranks = g_ranks.cpu().numpy()
    screened = 0
    for i, s in enumerate(o_scores):
        if (np.abs(s[1:] - s[0]) <= 1e-5).any():
            screened += 1
        else:
            assert g_ranks[i] == o_ranks[i], (i, g_ranks[i], o_ranks[i])
    assert screened <= len(o_scores) // 20
    if screened == 0:
        assert hits10 == pytest.approx(float((o_ranks <= 10).mean()), abs=0)
        assert mrr == pytest.approx(float((1.0 / o_ranks).mean()), rel=1e-12)
        assert hits5 == pytest.approx(float((o_ranks <= 5).mean()), abs=0)


def test_zsl_module_train_runs_gan_and_saves(tmp_path):
    from module.zsl_module import ZSLmodule
    g, root, args, ds, um = _setup(tmp_path, seed=6)
    zsl = ZSLmodule(args, root, ds.r2id, ds.e2id, DEV, ds)
    ent, rel = embeddings(g, 200, seed=7)
    zsl.update_embed(ent, rel)
    before = um.des_rel_map_layer1.weight_orig.detach().clone()
    ex_before = zsl.Extractor.fc1.weight.detach().clone()
    assert zsl.Extractor.training                       # as the reference's: train mode until eval()
    res = zsl.train(um)
    assert len(res) == 3 and all(0.0 <= float(x) <= 1.0 for x in res)
    assert not torch.equal(before, um.des_rel_map_layer1.weight_orig.detach())   # G was trained
    assert not torch.equal(ex_before, zsl.Extractor.fc1.weight.detach())         # the Extractor was pretrained
    assert len(zsl.pretrain_losses) == args.pretrain_times + 1 and np.all(np.isfinite(zsl.pretrain_losses))
    assert {"Generator", "Discriminator", "Extractor"} <= set(os.listdir(args.save_path))
    # after eval() the Extractor stays in eval mode: a second train() pretrains without dropout
    assert not zsl.Extractor.training
    zsl.train(um)
    # the saved Generator is the reference-layout UnifiedModel state dict
    sd = torch.load(os.path.join(args.save_path, "Generator"), weights_only=True)
    assert "layer_norm.a_2" in sd and not any(k.startswith("gen.") for k in sd)
    zsl.load(um)
    # nn.Module semantics stay available
    zsl.eval()
    zsl.train()


def test_main_training_cadence(tmp_path, monkeypatch):
    """main.main: edge batches -> repo NegativeSampling (GPU sampler + fused margin loss,
    gradients into the structure table and the relation branch's SN layers) -> Adam, and at
    save_epochs the checkpoint + generate_ent/rel_embed + ZSLmodule.train (GAN + eval)."""
    import main
    g = make_graph(seed=8)
    data_root = str(tmp_path / "origin_data")
    _write_dataset(os.path.join(data_root, "FB-synth"), g, 8)
    args = _args(str(tmp_path), dataset="FB-synth", epochs=2, save_epochs=2, train_times=2,
                 saved_model_name="unit")
    monkeypatch.chdir(tmp_path)
    out = main.main(args, data_root=data_root, save_root=str(tmp_path / "saved_models"), max_steps_per_epoch=6)
    assert len(out["losses"]) == 2 and all(np.isfinite(out["losses"]))
    assert os.path.exists(tmp_path / "saved_models" / "FB-synth" / "epoch2_unit.ckpt")
    assert os.path.exists(tmp_path / "saved_models" / "unit.ckpt")
    sd = torch.load(tmp_path / "saved_models" / "unit.ckpt", weights_only=True)
    assert "model.layer_norm.a_2" in sd and "ent_encoder.weight" in sd
    # the --evaluate branch on the checkpoint just written
    args.evaluate, args.pretrained_model_name = True, "epoch2_unit"
    res = main.run_evaluate(args, data_root=data_root, save_root=str(tmp_path / "saved_models"))
    assert len(res) == 3
