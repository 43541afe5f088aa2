"""Zero-shot relation-embedding generator (csrc/generator.hip), the MLP part of
UnifiedModel.generate (module/model.py:674-686): cat(noise, CLS) -> three spectral-normalised
Linear layers (module/spectral_norm.py) -> LayerNormalization (module/submodule.py:58-77).
The frozen M3AE text encoder that produces the CLS input is outside the hot path
(SURVEY.md §8(f)); callers pass the CLS rows in."""
from __future__ import annotations

import torch
import torch.nn as nn

from ._lib import call, lib, ptr, require_cuda, stream_ptr


class SNLinear(nn.Module):
    """Linear layer carrying spectral-norm state with the reference's state-dict names
    (weight_orig, weight_u, weight_v, bias; spectral_norm.py:129-137)."""

    def __init__(self, in_features: int, out_features: int, eps: float = 1e-12):
        super().__init__()
        lin = nn.Linear(in_features, out_features)
        self.weight_orig = nn.Parameter(lin.weight.detach().clone())
        self.bias = nn.Parameter(lin.bias.detach().clone())
        self.register_buffer("weight_u", nn.functional.normalize(torch.randn(out_features), dim=0, eps=eps))
        self.register_buffer("weight_v", nn.functional.normalize(torch.randn(in_features), dim=0, eps=eps))
        self.in_features, self.out_features, self.eps = in_features, out_features, eps


class RelationGenerator(nn.Module):
    """generate_fc_layer (in -> red), des_rel_map_layer1 (red -> D), des_rel_map_layer2 (D -> D),
    layer_norm (D): the exact module names of UnifiedModel (model.py:544-549, 554)."""

    def __init__(self, reduced_dim: int = 384, noise_dim: int = 15, emb_dim: int = 200, ln_eps: float = 1e-3):
        super().__init__()
        self.reduced_dim, self.noise_dim, self.dim = reduced_dim, noise_dim, emb_dim
        self.generate_fc_layer = SNLinear(reduced_dim + noise_dim, reduced_dim)
        self.des_rel_map_layer1 = SNLinear(reduced_dim, emb_dim)
        self.des_rel_map_layer2 = SNLinear(emb_dim, emb_dim)
        self.ln_a = nn.Parameter(torch.ones(emb_dim))
        self.ln_b = nn.Parameter(torch.zeros(emb_dim))
        self.ln_eps = ln_eps

    def forward(self, cls: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
        """cls (N, reduced_dim), noise (N, noise_dim) -> (N, emb_dim). In training mode one
        spectral-norm power iteration updates weight_u / weight_v in place first."""
        require_cuda(cls, noise)
        n = int(cls.shape[0])
        L0, L1, L2 = self.generate_fc_layer, self.des_rel_map_layer1, self.des_rel_map_layer2
        dev = cls.device
        out = torch.empty((n, self.dim), dtype=torch.float32, device=dev)
        work = torch.empty(int(lib().mmre_generator_workspace(n, L0.in_features, L0.out_features, L1.out_features,
                                                              L2.out_features)), dtype=torch.float32, device=dev)
        c = lambda t: t.detach().contiguous().float()
        noise_c, cls_c = c(noise), c(cls)
        ws = [c(L.weight_orig) for L in (L0, L1, L2)]
        bs = [c(L.bias) for L in (L0, L1, L2)]
        for L in (L0, L1, L2):
            if not (L.weight_u.is_contiguous() and L.weight_v.is_contiguous()):
                raise ValueError("spectral-norm buffers must be contiguous")
        call("mmre_generator_forward", ptr(noise_c), self.noise_dim, ptr(cls_c), self.reduced_dim, n,
             ptr(ws[0]), ptr(bs[0]), ptr(L0.weight_u), ptr(L0.weight_v), L0.out_features,
             ptr(ws[1]), ptr(bs[1]), ptr(L1.weight_u), ptr(L1.weight_v), L1.out_features,
             ptr(ws[2]), ptr(bs[2]), ptr(L2.weight_u), ptr(L2.weight_v), L2.out_features,
             ptr(c(self.ln_a)), ptr(c(self.ln_b)), float(self.ln_eps), int(self.training), float(L0.eps),
             ptr(out), ptr(work), stream_ptr(dev))
        return out

    def generate(self, cls: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
        """UnifiedModel.generate with the CLS already computed (model.py:679-686)."""
        return self.forward(cls, noise)
