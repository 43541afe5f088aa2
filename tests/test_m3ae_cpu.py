"""CPU checks of the M3AE text-encoder path: the host pieces (position
table, reference parameter names, state-dict loading), the oracle's padding
invariances -- the property the padding-free HIP path relies on -- and the C ABI exports and
argument checks (nothing is launched)."""
import ctypes

import numpy as np
import pytest
import torch

BLOCK_KEYS = ("layer_norm1.weight", "layer_norm1.bias", "attention.qkv_linear.weight", "attention.qkv_linear.bias",
              "attention.fc.weight", "attention.fc.bias", "layer_norm2.weight", "layer_norm2.bias",
              "transformer_mlp.fc1.weight", "transformer_mlp.fc1.bias", "transformer_mlp.fc2.weight",
              "transformer_mlp.fc2.bias")


def _encoder(vocab=50, depth=2, seed=0):
    from mmre.m3ae import M3AETextEncoder
    torch.manual_seed(seed)
    enc = M3AETextEncoder(vocab, 384, depth, 6)
    with torch.no_grad():
        for n, p in enc.named_parameters():
            if "layer_norm" in n:
                p.add_(0.1 * torch.randn_like(p))
    return enc


def test_pos_table_matches_reference_formula():
    import m3ae_text as om
    from mmre.m3ae import sincos_pos_embed_1d
    t = sincos_pos_embed_1d(384, 320)
    assert torch.equal(t, om.sincos_pos_embed_1d(384, 320)[0])
    pos = np.arange(320)[:, None].astype(np.float64)
    omega = 1.0 / 10000 ** (np.arange(192) / 192.0)
    ref = np.concatenate([np.sin(pos * omega), np.cos(pos * omega)], 1)
    assert np.abs(t.numpy() - ref).max() < 1e-4  # fp32 evaluation of model.py:113-133


def test_state_dict_names_follow_reference():
    enc = _encoder(depth=2)
    keys = set(enc.state_dict())
    expected = {"text_embedding.weight", "encoder_text_type_embedding", "cls_token", "encoder.layer_norm.weight",
                "encoder.layer_norm.bias"}
    expected |= {f"encoder.blocks.{i}.{k}" for i in range(2) for k in BLOCK_KEYS}
    assert keys == expected
    sd = enc.state_dict()
    assert sd["encoder.blocks.0.attention.qkv_linear.weight"].shape == (1152, 384)
    assert sd["encoder.blocks.1.transformer_mlp.fc1.weight"].shape == (1536, 384)
    assert sd["cls_token"].shape == (1, 1, 384)
    assert not any(p.requires_grad for p in enc.parameters())


def test_model_type_sizes():
    from mmre.m3ae import M3AETextEncoder
    e = M3AETextEncoder(10, model_type="tiny")
    assert (e.emb_dim, e.depth, e.num_heads) == (384, 2, 6)


def test_load_reference_state_dict_ignores_decoder():
    enc, other = _encoder(seed=0), _encoder(seed=1)
    full = dict(enc.state_dict())
    full["decoder.blocks.0.layer_norm1.weight"] = torch.ones(512)
    full["image_embedding.weight"] = torch.zeros(384, 768)
    other.load_reference_state_dict(full)
    for k, v in other.state_dict().items():
        assert torch.equal(v, full[k])
    del full["cls_token"]
    with pytest.raises(KeyError):
        other.load_reference_state_dict(full)


def test_oracle_padding_is_inert():
    """What the padding-free HIP path relies on: the CLS output does not depend on the token ids
    at padded positions (bit-identical: their softmax weights are exactly 0), and a right-padded
    row equals its truncation up to summation order."""
    import m3ae_text as om
    enc = _encoder(vocab=60, depth=2)
    sd = enc.state_dict()
    g = torch.Generator().manual_seed(3)
    L = 24
    tok = torch.randint(0, 60, (3, L), generator=g)
    msk = torch.zeros(3, L)
    msk[0, 10:] = 1
    msk[1, 3:7] = 1
    msk[1, 15:] = 1
    cls, _ = om.forward_representation_text(sd, tok, msk, 6)
    tok2 = torch.where(msk > 0, torch.randint(0, 60, (3, L), generator=g), tok)
    cls2, _ = om.forward_representation_text(sd, tok2, msk, 6)
    assert torch.equal(cls, cls2)
    short, _ = om.forward_representation_text(sd, tok[:1, :10], msk[:1, :10], 6)
    assert torch.allclose(short, cls[:1], atol=1e-5, rtol=0)


def test_m3ae_c_abi_exports_and_argument_checks():
    from mmre import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    for n in ("mmre_m3ae_max_len", "mmre_m3ae_plan_size", "mmre_m3ae_plan", "mmre_m3ae_workspace", "mmre_m3ae_encode",
              "mmre_m3ae_layernorm", "mmre_m3ae_linear", "mmre_m3ae_attention"):
        assert hasattr(L, n)
    lib = _lib.lib()
    assert lib.mmre_m3ae_max_len() >= 320
    assert lib.mmre_m3ae_workspace(100, 4, 384) == 100 * 384 * 10 + 4 * 384 * 7
    dummy = ctypes.c_void_p(16)
    # shape / argument errors come back as status codes before any launch
    assert lib.mmre_m3ae_linear(0, dummy, 10, 100, dummy, 384, dummy, None, dummy, None) == 3  # k % 32
    assert lib.mmre_m3ae_linear(0, dummy, 10, 384, dummy, 200, dummy, None, dummy, None) == 3  # n % 64
    assert lib.mmre_m3ae_linear(2, dummy, 10, 384, dummy, 384, dummy, None, dummy, None) == 1  # no residual
    assert lib.mmre_m3ae_layernorm(dummy, 4, 200, dummy, dummy, 1e-5, dummy, None) == 3
    assert lib.mmre_m3ae_attention(dummy, dummy, 2, 400, 6, 64, 0.125, 0, dummy, None) == 3  # rows > max
    assert lib.mmre_m3ae_attention(dummy, dummy, 2, 10, 6, 32, 0.125, 0, dummy, None) == 3  # head dim
    assert lib.mmre_m3ae_plan_size(10) == 65
    assert lib.mmre_m3ae_plan(dummy, dummy, 2, 400, 1, 10, dummy, None) == 1  # len > max_len
    params = (ctypes.c_void_p * 30)(*([16] * 30))
    assert lib.mmre_m3ae_encode(ctypes.cast(params, ctypes.c_void_p), 2, 200, 4, 1e-5, dummy, dummy, 1, 8, 10,
                                dummy, 1, 9, 9, dummy, 10 ** 6, dummy, None) == 3  # d = 200 unsupported
    assert lib.mmre_m3ae_encode(ctypes.cast(params, ctypes.c_void_p), 2, 384, 6, 1e-5, dummy, dummy, 2, 8, 10,
                                dummy, 3, 9, 9, dummy, 10 ** 6, dummy, None) == 1  # n_unique > n_seq


def test_encoder_needs_device_tensors():
    from mmre._lib import MMREError
    enc = _encoder()
    with pytest.raises(MMREError):
        enc.encode(torch.zeros((1, 4), dtype=torch.int32), torch.zeros((1, 4)))
