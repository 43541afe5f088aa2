"""Frozen M3AE text encoder (csrc/m3ae.hip): the producer of the generator's CLS input.

Replaces ``MaskedMultimodalAutoencoder.forward_representation(image=None, text,
text_padding_mask, deterministic=True)`` (module/model.py:323-356) over the Transformer of
module/submodule.py:128-238, as ``UnifiedModel.generate`` (model.py:674-679) and
``forward_relation_emb`` (model.py:599-604) call it under ``torch.no_grad`` (SURVEY.md §8(f)
rank 4). Parameter names are the reference's, so the encoder half of a reference M3AE state dict
loads with ``load_reference_state_dict`` (image / decoder tensors are ignored).

The encoder runs padding-free: only the CLS row and the unpadded tokens of each description
are computed (a padded key's logit is -1e7, its softmax weight exactly 0, and every other op
is row-wise), and the last block runs on the CLS rows alone. A description row equal to the
previous one (the reference repeats one description test_sample / G_batch_size times,
zsl_module.py:662-665, utils.py:686) is encoded once: the frozen encoder is a deterministic
function of the unpadded tokens, so deduplication is exact. There is no fallback: without libmmre_hip.so every
call raises.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from ._lib import MMREError, call, lib, ptr, require_cuda, stream_ptr

# module/utils.py:126-192, encoder side: (emb_dim, depth, num_heads)
MODEL_SIZES = {"small": (384, 12, 6), "small_modif": (384, 12, 6), "base": (768, 12, 12), "large": (1024, 24, 16),
               "huge": (1280, 32, 16), "debug": (1024, 2, 16), "tiny": (384, 2, 6), "tiny4": (384, 4, 6)}
LN_EPS = 1e-5  # nn.LayerNorm default (submodule.py:198, 201, 231)


def sincos_pos_embed_1d(embed_dim: int, length: int) -> torch.Tensor:
    """get_1d_sincos_pos_embed(embed_dim, length)[0] (model.py:113-133): (length, D) float32,
    evaluated with the reference's own torch CPU ops (a constant table, like a weight)."""
    omega = torch.arange(embed_dim // 2, dtype=torch.float32)
    omega /= embed_dim / 2.
    omega = 1. / 10000 ** omega
    pos = torch.arange(length, dtype=torch.float32).view(-1)
    out = torch.einsum("m,d->md", pos, omega)
    return torch.cat([torch.sin(out), torch.cos(out)], dim=1)


class _Attention(nn.Module):  # submodule.py:148-162, use_bias=True (Block, :199)
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.qkv_linear = nn.Linear(dim, dim * 3, bias=True)
        self.fc = nn.Linear(dim, dim)


class _TransformerMLP(nn.Module):  # submodule.py:128-138 (hidden = 4 dim, mlp_ratio unused)
    def __init__(self, dim):
        super().__init__()
        self.fc1 = nn.Linear(dim, 4 * dim)
        self.fc2 = nn.Linear(4 * dim, dim)


class _Block(nn.Module):  # submodule.py:188-203
    def __init__(self, dim, num_heads):
        super().__init__()
        self.layer_norm1 = nn.LayerNorm(dim)
        self.attention = _Attention(dim, num_heads)
        self.layer_norm2 = nn.LayerNorm(dim)
        self.transformer_mlp = _TransformerMLP(dim)


class _Transformer(nn.Module):  # submodule.py:216-231
    def __init__(self, dim, depth, num_heads):
        super().__init__()
        self.blocks = nn.ModuleList([_Block(dim, num_heads) for _ in range(depth)])
        self.layer_norm = nn.LayerNorm(dim)


class M3AETextEncoder(nn.Module):
    """The text branch of MaskedMultimodalAutoencoder (model.py:229-266 parameter names and
    init; model_type from the size table of utils.py:126-192). Frozen: no parameter requires
    grad (the reference calls it under torch.no_grad)."""

    def __init__(self, text_vocab_size: int, emb_dim: int = 384, depth: int = 12, num_heads: int = 6,
                 model_type: str | None = None):
        super().__init__()
        if model_type is not None:
            emb_dim, depth, num_heads = MODEL_SIZES[model_type]
        if text_vocab_size <= 0:
            raise ValueError("text_vocab_size must be positive")
        self.text_vocab_size = int(text_vocab_size)
        self.emb_dim, self.depth, self.num_heads = int(emb_dim), int(depth), int(num_heads)
        self.text_embedding = nn.Embedding(self.text_vocab_size, self.emb_dim)
        self.text_embedding.weight.data.normal_(0.0, 1.0)
        self.encoder_text_type_embedding = nn.Parameter(torch.empty(1, 1, self.emb_dim).normal_(0.02))
        self.cls_token = nn.Parameter(torch.empty(1, 1, self.emb_dim).normal_(0.02))
        self.encoder = _Transformer(self.emb_dim, self.depth, self.num_heads)
        for p in self.parameters():
            p.requires_grad_(False)
        self._pos = {}

    def load_reference_state_dict(self, sd):
        """Load the encoder tensors of a MaskedMultimodalAutoencoder state dict (model.py:200);
        decoder, image and mask-embedding entries are ignored, missing encoder entries raise."""
        own = self.state_dict()
        missing = [k for k in own if k not in sd]
        if missing:
            raise KeyError(f"state dict lacks encoder tensors: {missing[:4]}...")
        self.load_state_dict({k: sd[k] for k in own})

    def _pos_table(self, length: int, dev) -> torch.Tensor:
        key = (int(length), str(dev))
        t = self._pos.get(key)
        if t is None:
            t = self._pos[key] = sincos_pos_embed_1d(self.emb_dim, length).to(dev).contiguous()
        return t

    def param_list(self, length: int, dev):
        """Tensors in mmre_m3ae_encode's h_params order (include/mmre.h)."""
        ts = [self.text_embedding.weight, self._pos_table(max(int(length), 1), dev), self.encoder_text_type_embedding,
              self.cls_token]
        for b in self.encoder.blocks:
            a, m = b.attention, b.transformer_mlp
            ts += [b.layer_norm1.weight, b.layer_norm1.bias, a.qkv_linear.weight, a.qkv_linear.bias, a.fc.weight,
                   a.fc.bias, b.layer_norm2.weight, b.layer_norm2.bias, m.fc1.weight, m.fc1.bias, m.fc2.weight,
                   m.fc2.bias]
        ts += [self.encoder.layer_norm.weight, self.encoder.layer_norm.bias]
        out = []
        for t in ts:
            t = t.detach()
            if not (t.is_cuda and t.dtype == torch.float32):
                raise MMREError("M3AE encoder parameters must be float32 device tensors (call .to(device) first)")
            out.append(t.contiguous())
        return out

    @torch.no_grad()
    def encode(self, text: torch.Tensor, text_padding_mask: torch.Tensor, dedupe: bool = True) -> torch.Tensor:
        """CLS vectors (B, D) of description rows text (B, L) int token ids and
        text_padding_mask (B, L) float (> 0 = padding). dedupe: a row equal to the previous row
        on its unpadded tokens reuses that row's CLS (exact; the reference's repeats are
        adjacent, zsl_module.py:662-665)."""
        require_cuda(text, text_padding_mask)
        if text.dim() != 2 or tuple(text_padding_mask.shape) != tuple(text.shape):
            raise ValueError("text and text_padding_mask must both be (B, L)")
        B, L = (int(s) for s in text.shape)
        if L > int(lib().mmre_m3ae_max_len()):
            raise MMREError(f"description rows of {L} tokens exceed the encoder's {lib().mmre_m3ae_max_len()}")
        dev = text.device
        if B == 0:
            return torch.empty((0, self.emb_dim), dtype=torch.float32, device=dev)
        tok = text.to(torch.int32).contiguous()
        msk = text_padding_mask.to(torch.float32).contiguous()
        st = stream_ptr(dev)
        plan = torch.empty(int(lib().mmre_m3ae_plan_size(B)), dtype=torch.int32, device=dev)
        call("mmre_m3ae_plan", ptr(tok), ptr(msk), B, L, int(bool(dedupe)), self.text_vocab_size, ptr(plan), st)
        n_unique, n_rows, max_rows, n_bad = (int(v) for v in plan[3 * B + 1:3 * B + 5].cpu())  # sizes the encode
        if n_bad:
            raise MMREError(f"{n_bad} token ids outside [0, text_vocab_size) on unpadded positions")
        work = torch.empty(int(lib().mmre_m3ae_workspace(n_rows, n_unique, self.emb_dim)), dtype=torch.float32,
                           device=dev)
        out = torch.empty((B, self.emb_dim), dtype=torch.float32, device=dev)
        params = self.param_list(L, dev)
        arr = (ctypes.c_void_p * len(params))(*[t.data_ptr() for t in params])
        call("mmre_m3ae_encode", ctypes.cast(arr, ctypes.c_void_p), self.depth, self.emb_dim, self.num_heads, LN_EPS,
             ptr(tok), ptr(msk), B, L, self.text_vocab_size, ptr(plan), n_unique, n_rows, max_rows, ptr(work),
             work.numel(), ptr(out), st)
        return out

    def forward(self, text, text_padding_mask):
        return self.encode(text, text_padding_mask)

    def forward_representation(self, image, text, text_padding_mask, deterministic=True):
        """model.py:323-356 for image=None: returns (cls_x (B, 1, D), None). The full token
        sequence is not materialised (only its CLS row is ever consumed on this path)."""
        if image is not None:
            raise MMREError("the image branch of M3AE is outside this path (text descriptions only)")
        if not deterministic:
            raise MMREError("the frozen encoder runs deterministic=True (model.py:602, 677)")
        cls = self.encode(text, text_padding_mask)
        return cls.unsqueeze(1), None
