"""m3ae_text.py -- TEST INFRASTRUCTURE ONLY: oracle for the frozen M3AE text encoder.

Only ``tests/`` and bench.py's cpu_baseline leg import this module, as the checker; the product
package never does. A plain torch-fp32 (CPU) restatement, operation for operation, of

* ``get_1d_sincos_pos_embed`` (``module/model.py:113-133``);
* ``MaskedMultimodalAutoencoder.forward_representation`` with ``image=None``
  (``model.py:323-356``): cls token + (text_embedding + position + type embedding), padding
  mask with a 0 for the CLS column;
* ``Transformer`` / ``Block`` / ``Attention`` / ``TransformerMLP``
  (``module/submodule.py:128-238``), deterministic (dropout p = 0, drop-path off):
  LN1 -> qkv -> (q k^T) * hd^-0.5 -> where(mask > 0, -1e7) -> softmax -> . v -> fc, residual;
  LN2 -> fc1 -> gelu -> fc2, residual; final LN -- over the FULL padded sequence, as the
  reference computes it.

Parity status: **unpinned by reference fixtures**. The reference holds no M3AE golden vectors,
its checkpoint is absent, and running the reference's own Python is denied in this pipeline
(DESIGN.md §6), so this restatement -- written from the reference's source text -- is the
oracle. The product path (csrc/m3ae.hip) computes only the unpadded rows and, in the last
block, only the CLS rows (exact up to summation order: a masked logit's softmax weight is
exactly 0), so parity is by tolerance (1e-4).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def sincos_pos_embed_1d(embed_dim, length):
    """model.py:113-133: (1, length, D)."""
    omega = torch.arange(embed_dim // 2, dtype=torch.float32)
    omega /= embed_dim / 2.
    omega = 1. / 10000 ** omega
    pos = torch.arange(length, dtype=torch.float32).view(-1)
    out = torch.einsum("m,d->md", pos, omega)
    return torch.cat([torch.sin(out), torch.cos(out)], dim=1).unsqueeze(0)


def _attention(x, sd, pre, heads, padding_mask):  # submodule.py:164-186
    batch, n, channels = x.shape
    qkv = F.linear(x, sd[pre + "qkv_linear.weight"], sd[pre + "qkv_linear.bias"])
    qkv = qkv.view(batch, n, 3, heads, channels // heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    att = torch.matmul(q, k.transpose(-2, -1)) * (channels // heads) ** -0.5
    pm = padding_mask.unsqueeze(1).unsqueeze(1).expand(att.shape)
    att = torch.where(pm > 0, torch.tensor(-1e7), att)
    att = F.softmax(att, dim=-1)
    y = torch.matmul(att, v).permute(0, 2, 1, 3).reshape(batch, n, channels)
    return F.linear(y, sd[pre + "fc.weight"], sd[pre + "fc.bias"])


def _block(x, sd, pre, heads, padding_mask):  # submodule.py:205-214
    d = x.shape[-1]
    y = F.layer_norm(x, (d,), sd[pre + "layer_norm1.weight"], sd[pre + "layer_norm1.bias"])
    x = x + _attention(y, sd, pre + "attention.", heads, padding_mask)
    y = F.layer_norm(x, (d,), sd[pre + "layer_norm2.weight"], sd[pre + "layer_norm2.bias"])
    y = F.linear(y, sd[pre + "transformer_mlp.fc1.weight"], sd[pre + "transformer_mlp.fc1.bias"])
    y = F.gelu(y)
    y = F.linear(y, sd[pre + "transformer_mlp.fc2.weight"], sd[pre + "transformer_mlp.fc2.bias"])
    return x + y


def forward_representation_text(sd, text, text_padding_mask, heads):
    """model.py:323-356 (image=None) with the encoder state dict `sd` (reference key names).
    Returns (cls_x (B, 1, D), x (B, 1 + L, D))."""
    sd = {k: v.detach().float().cpu() for k, v in sd.items()}
    text = torch.as_tensor(text).long().cpu()
    mask = torch.as_tensor(text_padding_mask).float().cpu()
    batch, length = text.shape
    d = sd["cls_token"].shape[-1]
    cls = sd["cls_token"].expand(batch, 1, d)
    text_x = F.embedding(text, sd["text_embedding.weight"]) + sincos_pos_embed_1d(d, length) \
        + sd["encoder_text_type_embedding"]
    x = torch.cat([cls, text_x], dim=1)
    pm = torch.cat([torch.zeros((batch, 1), dtype=torch.float32), mask], dim=1)
    depth = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("encoder.blocks."))
    for i in range(depth):
        x = _block(x, sd, f"encoder.blocks.{i}.", heads, pm)
    x = F.layer_norm(x, (d,), sd["encoder.layer_norm.weight"], sd["encoder.layer_norm.bias"])
    return x[:, :1, :], x
