"""SGD whose plain step (no momentum, dampening, weight decay, nesterov or maximize) runs as one
HIP launch over every parameter tensor (mmre_sgd_step, csrc/optim.hip) -- the OpenKE Trainer's
default optimizer (Trainer.py:82-86, optim.SGD(parameters, lr, weight_decay)) after the fused
negative-sampling gradient. Any other configuration is torch.optim.SGD's own step."""
from __future__ import annotations

import ctypes

import torch

from ._lib import call, stream_ptr

_MAX_T = 8


class SGD(torch.optim.SGD):
    def _plain(self, group) -> bool:
        return (group["momentum"] == 0 and group["weight_decay"] == 0 and not group["nesterov"]
                and not group["maximize"])

    def _eligible(self, group, ps) -> bool:
        return self._plain(group) and all(
            p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and not p.grad.is_sparse
            and p.grad.dtype == torch.float32 and p.grad.is_contiguous()
            and p.data_ptr() % 16 == 0 and p.grad.data_ptr() % 16 == 0 for p in ps)  # float4 streams

    @torch.no_grad()
    def step(self, closure=None):
        work = []
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if ps and not self._eligible(group, ps):
                return super().step(closure)  # torch's own SGD step for every group
            work.append((group, ps))
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group, ps in work:
            lr = float(group["lr"])
            for i in range(0, len(ps), _MAX_T):
                chunk = ps[i:i + _MAX_T]
                n = len(chunk)
                params = (ctypes.c_void_p * n)(*[p.data_ptr() for p in chunk])
                grads = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in chunk])
                numel = (ctypes.c_int64 * n)(*[p.numel() for p in chunk])
                call("mmre_sgd_step", ctypes.cast(params, ctypes.c_void_p), ctypes.cast(grads, ctypes.c_void_p),
                     ctypes.cast(numel, ctypes.c_void_p), n, lr, stream_ptr(chunk[0].device))
        return loss
