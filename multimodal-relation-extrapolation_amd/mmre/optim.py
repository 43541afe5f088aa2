"""SGD whose plain step (no momentum, dampening, weight decay, nesterov or maximize) runs as one
HIP launch over every parameter tensor (mmre_sgd_step, csrc/optim.hip) -- the OpenKE Trainer's
default optimizer (Trainer.py:82-86, optim.SGD(parameters, lr, weight_decay)) after the fused
negative-sampling gradient. Any other configuration is torch.optim.SGD's own step; such steps
are counted in SGD.fallback_steps (reason in SGD.fallback_reason), so a run can show that the
HIP step was the one that ran."""
from __future__ import annotations

import ctypes

import torch

from ._lib import call, mark_written, stream_ptr

_MAX_T = 8


class SGD(torch.optim.SGD):
    def _plain(self, group) -> bool:
        return (group["momentum"] == 0 and group["weight_decay"] == 0 and not group["nesterov"]
                and not group["maximize"])

    def _eligible(self, group, ps) -> bool:
        return self._why_not(group, ps) is None

    # steps that took torch's own SGD path instead of mmre_sgd_step, and why (last reason)
    fallback_steps = 0
    fallback_reason = None

    # ---- fused mode: the fused negative-sampling backward applies this optimizer's step to the
    # embedding tables in its row-owner pass (mmre.ns.fused_ns_loss(..., optimizer=opt)); step()
    # then skips them. Bit-identical parameters (same fma), one pass over the tables fewer.
    # Guards: a table is fused only when EVERY group of the optimizer takes the HIP
    # step (so step() never falls back to torch's step over parameters it already updated), no
    # gradient exists yet and no fused step of the table is pending; a gradient that reaches a
    # fused table after its fused step (a second backward before step(): gradient accumulation)
    # makes step() raise instead of silently dropping it; zero_grad() clears the pending state.
    def fusable_lr(self, tables):
        """lr when `tables` can take the fused step: all in one plain group, eligible for the HIP
        step, every other group plain too, without a gradient yet (autograd will assign theirs,
        not accumulate) and not already fused since the last step(); else None."""
        ids = {id(t) for t in tables}
        if ids & set(getattr(self, "_fused_done", {})):
            return None
        if any(not self._plain(g) for g in self.param_groups):
            return None
        for group in self.param_groups:
            mine = [p for p in group["params"] if id(p) in ids]
            if not mine:
                continue
            if len(mine) != len(ids) or any(p.grad is not None or not p.requires_grad or not p.is_leaf for p in mine):
                return None
            if float(group["lr"]) == 0.0:
                return None
            if any(not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous() for p in mine):
                return None
            for t in mine:  # before the backward that will fuse: its own accumulation is then seen too
                hooked = getattr(t, "_mmre_fuse_hooks", None)
                if hooked is None:
                    hooked = t._mmre_fuse_hooks = set()
                if id(self) not in hooked:
                    t.register_post_accumulate_grad_hook(self._count_accumulation)
                    hooked.add(id(self))
            return float(group["lr"])
        return None

    def _fused_applied(self, tables):
        """Called by the fused backward once it has updated `tables`: step() skips them. The
        gradient autograd assigns next is the fused one; any later accumulation into it marks
        the table dirty (post-accumulate-grad hook), and step() then raises."""
        if not hasattr(self, "_fused_done"):
            self._fused_done = {}
        for t in tables:
            self._fused_done[id(t)] = 0  # accumulations seen since the fused backward (hook: fusable_lr)

    def _count_accumulation(self, p):
        done = getattr(self, "_fused_done", None)
        if done is not None and id(p) in done:
            done[id(p)] += 1

    def zero_grad(self, set_to_none: bool = True):
        self._fused_done = {}
        super().zero_grad(set_to_none=set_to_none)

    def _why_not(self, group, ps):
        if not self._plain(group):
            return "momentum / weight_decay / nesterov / maximize"
        for p in ps:
            if not p.is_cuda or p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                return "not a float32 device tensor"
            if p.grad.is_sparse:
                return "sparse gradient"
            if not p.is_contiguous() or not p.grad.is_contiguous():
                return "non-contiguous parameter or gradient"
            if p.data_ptr() % 16 or p.grad.data_ptr() % 16:
                return "parameter or gradient not 16-B aligned (float4 streams)"
        return None

    @torch.no_grad()
    def step(self, closure=None):
        # torch.optim.SGD's order: the closure first (it may create or refresh the gradients),
        # then the parameters that have one
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        done = getattr(self, "_fused_done", {})
        self._fused_done = {}
        late = [k for k, c in done.items() if c > 1]  # the fused backward's own assignment counts once
        if late:
            raise RuntimeError("mmre.optim.SGD: a table whose SGD step the fused backward already applied received "
                               "more gradient before step() (e.g. gradient accumulation); call zero_grad() between "
                               "backward passes or build the loss without optimizer= (mmre.ns.fused_ns_loss)")
        work = []
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None and id(p) not in done]
            why = self._why_not(group, ps) if ps else None
            if why is not None:  # torch's own SGD step -- counted, not silent -- over what was not fused
                type(self).fallback_steps += 1
                type(self).fallback_reason = why
                fused = [p for g in self.param_groups for p in g["params"] if id(p) in done]
                saved = [p.grad for p in fused]
                for p in fused:
                    p.grad = None  # torch's step skips parameters without a gradient
                try:
                    super().step()
                finally:
                    for p, g in zip(fused, saved):
                        p.grad = g
                return loss
            work.append((group, ps))
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
                mark_written(*chunk)  # as torch's in-place SGD update would
        return loss
