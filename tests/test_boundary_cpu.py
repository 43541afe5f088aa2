"""The repo-level drop-in surface on CPU: UnifiedModel's state-dict
layout is the reference's (module/model.py:517-555), each key once; a reference-layout
checkpoint loads with strict=True (out-of-path tensors carried and written back); the dataset
mirror, the edge-batch sampler and the args surface. No kernel is launched."""
import json
import os
from types import SimpleNamespace as NS

import numpy as np
import pytest
import torch

from zsl_synth import make_graph


def _args(**kw):
    from args import read_options
    a = read_options([])
    a.model_type = "tiny"
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _dataset(vocab=500, nodes=50):
    return NS(vocab_size=vocab, num_nodes=nodes,
              config=NS(image_only=False, text_only=False, tokenizer_max_length=320, unpaired_tokenizer_max_length=320,
                        struct_only=False))


# model.py:544-555 + spectral_norm.py:129-137 (weight_orig parameter, weight_u / weight_v buffers)
REFERENCE_GENERATOR_KEYS = {f"{layer}.{p}" for layer in ("des_rel_map_layer1", "des_rel_map_layer2", "generate_fc_layer")
                            for p in ("weight_orig", "bias", "weight_u", "weight_v")} | {"layer_norm.a_2",
                                                                                          "layer_norm.b_2"}


def _reference_layout_state(m, rng):
    """A state dict keyed like the reference UnifiedModel's: the generator part with new values,
    plus RGCN conv (num_bases 30, model.py:552) and M3AE image / decoder tensors."""
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for k in REFERENCE_GENERATOR_KEYS:
        sd[k] = torch.from_numpy(rng.standard_normal(tuple(sd[k].shape)).astype(np.float32))
    R, red, d = m.num_relations, m.reduced_dim, m.dim
    sd.update({"conv.weight": torch.randn(30, red, d), "conv.comp": torch.randn(R, 30), "conv.root": torch.randn(red, d),
               "conv.bias": torch.randn(d), "M3AEmodel.image_embedding.weight": torch.randn(red, 768),
               "M3AEmodel.image_embedding.bias": torch.randn(red), "M3AEmodel.decoder.layer_norm.weight": torch.randn(512),
               "M3AEmodel.decoder_text_output.weight": torch.randn(500, 512),
               "M3AEmodel.image_mask_embedding": torch.randn(1, 1, 512)})
    return sd


def test_unified_model_keys_are_the_reference_keys_once():
    from module.model import UnifiedModel
    m = UnifiedModel(_args(), 200, _dataset(), 12, 15)
    keys = list(m.state_dict().keys())
    assert len(keys) == len(set(keys))
    gen = {k for k in keys if not k.startswith("M3AEmodel.")}
    assert gen == REFERENCE_GENERATOR_KEYS
    assert not any(k.startswith("gen.") or "ln_a" in k or "ln_b" in k for k in keys)
    # the GAN step's generator view shares the same tensors (no copy, no second registration)
    assert m.generator.ln_a is m.layer_norm.a_2
    assert m.generator.generate_fc_layer.weight_orig is m.generate_fc_layer.weight_orig


def test_reference_checkpoint_loads_strict_and_round_trips():
    from module.model import UnifiedModel
    m = UnifiedModel(_args(), 200, _dataset(), 12, 15)
    sd = _reference_layout_state(m, np.random.default_rng(0))
    res = m.load_state_dict(sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    for k in REFERENCE_GENERATOR_KEYS:
        torch.testing.assert_close(m.state_dict()[k], sd[k], rtol=0, atol=0)
    torch.testing.assert_close(m.generator.ln_a.detach(), sd["layer_norm.a_2"], rtol=0, atol=0)
    out = m.state_dict()
    assert set(out) == set(sd)               # carried tensors are written back
    torch.testing.assert_close(out["conv.comp"], sd["conv.comp"], rtol=0, atol=0)
    m2 = UnifiedModel(_args(), 200, _dataset(), 12, 15)
    m2.load_state_dict(out, strict=True)
    bad = dict(sd, **{"not_a_reference_key.weight": torch.zeros(1)})
    with pytest.raises(RuntimeError):
        m2.load_state_dict(bad, strict=True)
    missing = {k: v for k, v in sd.items() if k != "layer_norm.b_2"}
    with pytest.raises(RuntimeError):
        m2.load_state_dict(missing, strict=True)


def _data_dir(tmp_path, g):
    d = tmp_path / "ds"
    d.mkdir()
    (d / "entity2ids_zsl.json").write_text(json.dumps(g["ent2id"]))
    (d / "relation2ids.json").write_text(json.dumps(g["rel2id"]))
    n_rel = max(g["rel2id"].values()) + 1
    (d / "rel_description_zsl").write_text("\n".join(f"relation {i}: a description, with words." * (1 + i % 3)
                                                     for i in range(n_rel)) + "\n")
    (d / "train_tasks_zsl.json").write_text(json.dumps(g["train_tasks"]))
    return str(d)


def test_zs_dataset_and_edge_batches(tmp_path):
    import main
    from module.data import ZSDataset
    g = make_graph(seed=3)
    ds = ZSDataset(_data_dir(tmp_path, g), max_len=64)
    assert ds.num_nodes == max(g["ent2id"].values()) + 1
    assert ds.rel_tokens.shape == (ds.num_relations, 64)
    assert torch.all((ds.rel_tokens == 0) == (ds.rel_mask == 1.0))
    b = ds.generate_batch([], torch.tensor([2, 0, 2]))
    assert torch.equal(b["rel_des"][0], b["rel_des"][2]) and b["image"].numel() == 0
    n_edges = ds.edge_index.shape[1]
    assert n_edges == sum(len(v) for v in g["train_tasks"].values())
    loader = main.EdgeBatches(ds.edge_index, ds.edge_type, ds.num_nodes, batch_size=12, sample_size=4, seed=0)
    seen = 0
    src, dst = ds.edge_index.numpy()
    for n_id, ei, et in loader:
        assert ei.shape[1] == len(et)
        seeds = set(n_id[:12].tolist())
        assert all(int(n_id[j]) in seeds for j in ei[1])             # targets are seed nodes
        per_seed = np.bincount(ei[1], minlength=len(n_id))
        assert per_seed.max(initial=0) <= 4
        glob = set(zip(src.tolist(), dst.tolist()))
        assert all((int(n_id[a]), int(n_id[b])) in glob for a, b in ei.T)
        seen += ei.shape[1]
    assert 0 < seen <= n_edges


def test_args_surface():
    from args import read_options
    a = read_options(["--evaluate", "--emb_dim", "256", "--dataset", "DB15K-ZS"])
    assert a.evaluate and a.emb_dim == 256 and a.save_path == "./origin_data/DB15K-ZS/Embed_used"
    assert (a.noise_dim, a.test_sample, a.max_neighbor, a.G_batch_size, a.gan_batch_rela) == (15, 20, 50, 256, 2)
