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
