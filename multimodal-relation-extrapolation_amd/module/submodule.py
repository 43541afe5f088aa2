"""BaseModule and LayerNormalization (module/submodule.py:7-77).

LayerNormalization is mmre.generator's (parameters a_2 / b_2, unbiased std, eps added to the
std, identity when z.size(1) == 1): a HIP kernel standalone, fused into the generator kernel
inside the relation generator (csrc/generator.hip)."""
import torch
import torch.nn as nn

from mmre.generator import LayerNormalization  # noqa: F401  (submodule.py:58-77, HIP forward)
from openke.module.BaseModule import BaseModule as _OKBase


class BaseModule(_OKBase):
    def load_checkpoint(self, path, device=None):
        super().load_checkpoint(path, map_location=device)


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
