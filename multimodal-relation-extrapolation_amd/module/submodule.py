"""BaseModule and LayerNormalization (module/submodule.py:7-77).

LayerNormalization here is the standalone module (device tensor ops) with the reference's
semantics -- unbiased std, eps added to the std, identity when z.size(1) == 1; inside the
relation generator it is fused into the HIP kernel (csrc/generator.hip)."""
import torch
import torch.nn as nn

from openke.module.BaseModule import BaseModule as _OKBase


class BaseModule(_OKBase):
    def load_checkpoint(self, path, device=None):
        super().load_checkpoint(path, map_location=device)


class LayerNormalization(nn.Module):
    def __init__(self, d_hid, eps=1e-3):
        super().__init__()
        self.eps = eps
        self.a_2 = nn.Parameter(torch.ones(d_hid), requires_grad=True)
        self.b_2 = nn.Parameter(torch.zeros(d_hid), requires_grad=True)

    def forward(self, z):
        if z.size(1) == 1:
            return z
        mu = torch.mean(z, keepdim=True, dim=-1)
        sigma = torch.std(z, keepdim=True, dim=-1)
        ln_out = (z - mu.expand_as(z)) / (sigma.expand_as(z) + self.eps)
        return ln_out * self.a_2.expand_as(ln_out) + self.b_2.expand_as(ln_out)


class SupportEncoder(nn.Module):
    """SupportEncoder (module/submodule.py:240-258): LayerNorm(proj2(relu(proj1(x))) + x),
    nn.LayerNorm (eps 1e-5, biased variance). Same parameter names and init (xavier_normal_
    weights). In eval mode forward runs on the GPU through the Extractor's fused MFMA kernel
    (csrc/extractor.hip) -- it is that kernel's per-row stage; training mode (dropout) is not
    part of this build."""

    def __init__(self, d_model, d_inner, dropout=0.1):
        super().__init__()
        self.proj1 = nn.Linear(d_model, d_inner)
        self.proj2 = nn.Linear(d_inner, d_model)
        self.layer_norm = nn.LayerNorm(d_model)
        nn.init.xavier_normal_(self.proj1.weight)
        nn.init.xavier_normal_(self.proj2.weight)
        self.dropout = nn.Dropout(dropout)
        self.relu = nn.ReLU()

    def forward(self, x):
        from mmre.extractor import support_encode
        return support_encode(self, x)
