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


class LayerNormalization(nn.Module):
    """LayerNormalization (module/submodule.py:58-77): parameters a_2 / b_2, unbiased std, eps
    added to the std, identity when z.size(1) == 1. Standalone calls run the HIP kernel
    (mmre.gemm.layer_norm, differentiable); inside the generator it is fused into
    csrc/generator.hip."""

    def __init__(self, d_hid: int, eps: float = 1e-3):
        super().__init__()
        self.eps = eps
        self.a_2 = nn.Parameter(torch.ones(d_hid), requires_grad=True)
        self.b_2 = nn.Parameter(torch.zeros(d_hid), requires_grad=True)

    def forward(self, z):
        from .gemm import layer_norm
        return layer_norm(self, z)


class RelationGenerator(nn.Module):
    """generate_fc_layer (in -> red), des_rel_map_layer1 (red -> D), des_rel_map_layer2 (D -> D),
    layer_norm (D): the module names, and so the state-dict keys, of UnifiedModel
    (model.py:544-549, 555): *.weight_orig / weight_u / weight_v / bias, layer_norm.a_2 / b_2."""

    def __init__(self, reduced_dim: int = 384, noise_dim: int = 15, emb_dim: int = 200, ln_eps: float = 1e-3):
        super().__init__()
        self.reduced_dim, self.noise_dim, self.dim = reduced_dim, noise_dim, emb_dim
        self.generate_fc_layer = SNLinear(reduced_dim + noise_dim, reduced_dim)
        self.des_rel_map_layer1 = SNLinear(reduced_dim, emb_dim)
        self.des_rel_map_layer2 = SNLinear(emb_dim, emb_dim)
        self.layer_norm = LayerNormalization(emb_dim, eps=ln_eps)

    @property
    def ln_a(self):
        return self.layer_norm.a_2

    @property
    def ln_b(self):
        return self.layer_norm.b_2

    @property
    def ln_eps(self):
        return float(self.layer_norm.eps)

    def forward(self, cls: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
        """cls (N, reduced_dim), noise (N, noise_dim) -> (N, emb_dim). In training mode one
        spectral-norm power iteration updates weight_u / weight_v in place first. With autograd
        recording and trainable parameters, the output carries the HIP backward
        (mmre_generator_backward) to weight_orig / bias / layer-norm a, b."""
        require_cuda(cls, noise)
        params = self._params()
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _GeneratorFn.apply(cls, noise, self, *params)
        return self._run(cls, noise)

    def _params(self):
        L0, L1, L2 = self.generate_fc_layer, self.des_rel_map_layer1, self.des_rel_map_layer2
        return [L0.weight_orig, L0.bias, L1.weight_orig, L1.bias, L2.weight_orig, L2.bias, self.ln_a, self.ln_b]

    def _run(self, cls, noise, acts=None):
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
        call("mmre_generator_forward_save", ptr(noise_c), self.noise_dim, ptr(cls_c), self.reduced_dim, n,
             ptr(ws[0]), ptr(bs[0]), ptr(L0.weight_u), ptr(L0.weight_v), L0.out_features,
             ptr(ws[1]), ptr(bs[1]), ptr(L1.weight_u), ptr(L1.weight_v), L1.out_features,
             ptr(ws[2]), ptr(bs[2]), ptr(L2.weight_u), ptr(L2.weight_v), L2.out_features,
             ptr(c(self.ln_a)), ptr(c(self.ln_b)), float(self.ln_eps), int(self.training), float(L0.eps),
             ptr(out), ptr(work), ptr(acts), stream_ptr(dev))
        if acts is not None:
            return out, work[3 * 2048:3 * 2048 + 3].clone()
        return out

    def generate(self, cls: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
        """UnifiedModel.generate with the CLS already computed (model.py:679-686)."""
        return self.forward(cls, noise)


class _GeneratorFn(torch.autograd.Function):
    """Generator forward (training form: activations kept) + its HIP backward. u, v and sigma
    are the values this forward used (cloned: a later forward updates u, v in place, as the
    reference's spectral_norm.py:74-85 clones them for the same reason)."""

    @staticmethod
    def forward(ctx, cls, noise, gen, w0, b0, w1, b1, w2, b2, ln_a, ln_b):
        n = int(cls.shape[0])
        L0, L1, L2 = gen.generate_fc_layer, gen.des_rel_map_layer1, gen.des_rel_map_layer2
        in0 = L0.in_features
        acts = torch.empty(int(lib().mmre_generator_acts_size(n, in0, L0.out_features, L1.out_features,
                                                              L2.out_features)), dtype=torch.float32, device=cls.device)
        out, sigma = gen._run(cls, noise, acts=acts)
        uv = [t.detach().clone() for L in (L0, L1, L2) for t in (L.weight_u, L.weight_v)]
        ctx.gen_dims = (n, in0, L0.out_features, L1.out_features, L2.out_features, float(gen.ln_eps))
        ctx.save_for_backward(acts, sigma, w0, w1, w2, ln_a, *uv)
        return out

    @staticmethod
    def backward(ctx, gout):
        acts, sigma, w0, w1, w2, ln_a, u0, v0, u1, v1, u2, v2 = ctx.saved_tensors
        n, in0, o0, o1, o2, eps = ctx.gen_dims
        dev = gout.device
        c = lambda t: t.detach().contiguous().float()
        g = [torch.empty_like(w0), torch.empty(o0, device=dev), torch.empty_like(w1), torch.empty(o1, device=dev),
             torch.empty_like(w2), torch.empty(o2, device=dev), torch.empty(o2, device=dev),
             torch.empty(o2, device=dev)]
        work = torch.empty(int(lib().mmre_generator_backward_workspace(n, in0, o0, o1, o2)), dtype=torch.float32,
                           device=dev)
        call("mmre_generator_backward", ptr(c(gout)), n, in0, o0, o1, o2, ptr(acts), ptr(sigma), ptr(c(w0)),
             ptr(u0), ptr(v0), ptr(c(w1)), ptr(u1), ptr(v1), ptr(c(w2)), ptr(u2), ptr(v2), ptr(c(ln_a)), eps,
             *[ptr(t) for t in g], ptr(work), stream_ptr(dev))
        return (None, None, None, *g)
