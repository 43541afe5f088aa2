"""Differentiable small fp32 matmul on the HIP kernel of csrc/gemm.hip.

The GAN step's Discriminator (module/zsl_module.py:112-138) multiplies 200-512-sided matrices:
x W^T of its spectral-normalised layers and the class scores against the centroids, then their
gradients, including the gradient penalty's double backward (module/utils.py:692-707). A
library GEMM runs each of those products on a single workgroup; `mm` cuts the output into
32 x 32 MFMA tiles and splits K across waves (deterministic slice-order sum). Its backward is
written with `mm` itself, so it is differentiable again (create_graph=True works). Any-stride
operands: transposes are passed as views, never copied.
"""
from __future__ import annotations

import torch

from ._lib import MMREError, call, lib, ptr, require_cuda, stream_ptr


def mm_hip(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a (M, K) @ b (K, N) -> (M, N) float32, on the device, no autograd."""
    require_cuda(a, b)
    if a.dtype != torch.float32 or b.dtype != torch.float32 or a.dim() != 2 or b.dim() != 2:
        raise MMREError("mm takes 2-d float32 device tensors")
    M, K = (int(s) for s in a.shape)
    K2, N = (int(s) for s in b.shape)
    if K != K2:
        raise MMREError(f"mm: inner dimensions differ ({K} vs {K2})")
    out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    S = int(lib().mmre_gemm_splits(M, N, K))
    work = torch.empty(S * M * N if S > 1 else 1, dtype=torch.float32, device=a.device)
    call("mmre_gemm_f32", ptr(a), a.stride(0), a.stride(1), ptr(b), b.stride(0), b.stride(1), M, N, K, ptr(work),
         work.numel(), ptr(out), stream_ptr(a.device))
    return out


class _MM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return mm_hip(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = mm(g, b.t()) if ctx.needs_input_grad[0] else None
        gb = mm(a.t(), g) if ctx.needs_input_grad[1] else None
        return ga, gb


def mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b with autograd (any order of derivatives)."""
    return _MM.apply(a, b)


def sn_linear(mod, x: torch.Tensor) -> torch.Tensor:
    """mod(x) for a spectral-normalised nn.Linear (torch.nn.utils.spectral_norm): its forward
    pre-hook first (the power iteration in training mode, weight = weight_orig / sigma), then
    x W^T + b with `mm` (F.linear's order: product, then bias)."""
    for hook in mod._forward_pre_hooks.values():
        hook(mod, (x,))
    return mm(x, mod.weight.t()) + mod.bias
