"""Differentiable pieces of the ZSL GAN Discriminator on HIP kernels (csrc/gemm.hip,
csrc/generator.hip).

The Discriminator (module/zsl_module.py:112-138) is a chain of small ops on 200-512-sided
matrices, run as torch autograd inside the GAN step's hipGraph; each torch op is a launch of
its own (~5 us each at these sizes), so the cost is the number of launches:

* `mm` -- products on the split-K GEMM: a library GEMM runs each of these on a single
  workgroup; here 32 x 32 MFMA tiles with K split over the waves of a workgroup (slice-order
  sum, deterministic), bias in the epilogue. Its backward is written with `mm` itself, so it is
  differentiable again (the gradient penalty's create_graph=True, module/utils.py:692-707).
  Any-stride operands: transposes are passed as views, never copied.
* `sn_weight` -- spectral_norm's compute_weight (spectral_norm.py:39-89) in one launch (power
  iteration, sigma, W / sigma, the u, v snapshot) instead of ~15 torch launches, and its
  backward (the SN chain rule) in one more.
* `layer_norm` -- LayerNormalization (module/submodule.py:58-77) forward in one launch; its
  backward is one row kernel + two column sums, or -- when a higher-order graph is being
  built (create_graph) -- the same formula in differentiable torch ops.
"""
from __future__ import annotations

import torch
from torch.autograd.function import once_differentiable
from torch.nn.utils.spectral_norm import SpectralNorm

from ._lib import MMREError, call, lib, ptr, require_cuda, stream_ptr


def mm_hip(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """a (M, K) @ b (K, N) (+ bias (N)) -> (M, N) float32, on the device, no autograd."""
    require_cuda(a, b, bias)
    if a.dtype != torch.float32 or b.dtype != torch.float32 or a.dim() != 2 or b.dim() != 2:
        raise MMREError("mm takes 2-d float32 device tensors")
    M, K = (int(s) for s in a.shape)
    K2, N = (int(s) for s in b.shape)
    if K != K2:
        raise MMREError(f"mm: inner dimensions differ ({K} vs {K2})")
    if bias is not None:
        if bias.dtype != torch.float32 or bias.numel() != N:
            raise MMREError("mm: bias must be float32 with N elements")
        bias = bias.contiguous()
    out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    call("mmre_gemm_f32", ptr(a), a.stride(0), a.stride(1), ptr(b), b.stride(0), b.stride(1), M, N, K, ptr(bias),
         ptr(out), stream_ptr(a.device))
    return out


class _MM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, bias):
        ctx.save_for_backward(a, b)
        ctx.has_bias = bias is not None
        return mm_hip(a, b, bias)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = mm(g, b.t()) if ctx.needs_input_grad[0] else None
        gb = mm(a.t(), g) if ctx.needs_input_grad[1] else None
        gbias = g.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return ga, gb, gbias


def mm(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """a @ b (+ bias) with autograd (any order of derivatives)."""
    return _MM.apply(a, b, bias)


class _SNWeight(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w, u, v, power_iteration, eps):
        out, inn = (int(s) for s in w.shape)
        dev = w.device
        w = w.detach().contiguous()
        sigma = torch.empty(1, dtype=torch.float32, device=dev)
        u_s, v_s = torch.empty_like(u), torch.empty_like(v)
        w_hat = torch.empty_like(w)
        work = torch.empty(2048, dtype=torch.float32, device=dev)
        call("mmre_sn_weight", ptr(w), out, inn, ptr(u), ptr(v), int(bool(power_iteration)), float(eps), ptr(sigma),
             ptr(u_s), ptr(v_s), ptr(w_hat), ptr(work), stream_ptr(dev))
        ctx.save_for_backward(w, u_s, v_s, sigma)
        return w_hat

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        w, u_s, v_s, sigma = ctx.saved_tensors
        gw = torch.empty_like(w)
        call("mmre_sn_weight_backward", ptr(g.contiguous()), ptr(w), int(w.shape[0]), int(w.shape[1]), ptr(u_s),
             ptr(v_s), ptr(sigma), ptr(gw), stream_ptr(w.device))
        return gw, None, None, None, None


def _sn_eps(mod) -> float:
    """eps of a spectral-normalised layer: a torch.nn.utils.spectral_norm hook (n_power_iterations
    1, dim 0, on 'weight') or mmre.generator.SNLinear's own state (same parameter names)."""
    for hook in mod._forward_pre_hooks.values():
        if isinstance(hook, SpectralNorm):
            if hook.n_power_iterations != 1 or hook.dim != 0 or hook.name != "weight":
                raise MMREError("sn_weight: spectral_norm with n_power_iterations=1, dim=0 on 'weight' only")
            return float(hook.eps)
    if all(hasattr(mod, a) for a in ("weight_orig", "weight_u", "weight_v", "eps")):
        return float(mod.eps)
    raise MMREError(f"{type(mod).__name__} is not spectral-normalised")


def sn_weight(mod) -> torch.Tensor:
    """W_orig / sigma of a spectral-normalised layer, as spectral_norm's forward pre-hook
    computes it (one power iteration on weight_u / weight_v in training mode,
    spectral_norm.py:74-89), in one launch."""
    eps = _sn_eps(mod)
    w = mod.weight_orig
    require_cuda(w)
    if w.dim() != 2:
        raise MMREError("sn_weight: 2-d weights only")
    return _SNWeight.apply(w, mod.weight_u, mod.weight_v, mod.training, eps)


def sn_linear(mod, x: torch.Tensor) -> torch.Tensor:
    """mod(x) for a spectral-normalised nn.Linear: x (W_orig / sigma)^T + b."""
    return mm(x, sn_weight(mod).t(), mod.bias)


def _ln_backward_torch(g, z, a, eps):
    """LayerNormalization's backward as differentiable torch ops (for create_graph)."""
    D = z.shape[1]
    c = z - z.mean(1, keepdim=True)
    sd = ((c * c).sum(1, keepdim=True) / (D - 1)).sqrt()
    d = sd + eps
    ga = g * a
    gz = (ga - ga.mean(1, keepdim=True)) / d - c * ((ga * c).sum(1, keepdim=True) / (d * d * sd * (D - 1)))
    return gz, (g * (c / d)).sum(0), g.sum(0)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, a, b, eps):
        z = z.contiguous()
        n, D = (int(s) for s in z.shape)
        out = torch.empty_like(z)
        call("mmre_layernorm_unbiased", ptr(z), n, D, ptr(a.contiguous()), ptr(b.contiguous()), float(eps), ptr(out),
             stream_ptr(z.device))
        ctx.save_for_backward(z, a)
        ctx.eps = float(eps)
        return out

    @staticmethod
    def backward(ctx, g):
        z, a = ctx.saved_tensors
        if torch.is_grad_enabled():  # building a higher-order graph: differentiable form
            return (*_ln_backward_torch(g, z, a, ctx.eps), None)
        n, D = (int(s) for s in z.shape)
        gz = torch.empty_like(z)
        ga = torch.empty(D, dtype=torch.float32, device=z.device)
        gb = torch.empty_like(ga)
        work = torch.empty_like(z)
        call("mmre_layernorm_unbiased_backward", ptr(g.contiguous()), ptr(z), n, D, ptr(a.contiguous()), ctx.eps,
             ptr(gz), ptr(ga), ptr(gb), ptr(work), stream_ptr(z.device))
        return gz, ga, gb, None


def layer_norm(mod, z: torch.Tensor) -> torch.Tensor:
    """module.submodule.LayerNormalization(z) (unbiased std, eps added to the std; identity when
    z.size(1) == 1) on the HIP kernel."""
    if z.size(1) == 1:
        return z
    require_cuda(z)
    if z.dim() != 2 or z.dtype != torch.float32:
        raise MMREError("layer_norm: 2-d float32 input")
    return _LayerNorm.apply(z, mod.a_2, mod.b_2, mod.eps)


def gemm_splits(m: int, n: int, k: int) -> int:
    """K slices (waves per output tile) the GEMM uses for an (m, n, k) product."""
    return int(lib().mmre_gemm_splits(m, n, k))
