"""Fused negative-sampling margin loss (csrc/ns.hip) as a torch.autograd.Function.

forward  = model(data) in 'normal' mode for B*(1+k) rows -> MarginLoss (optionally
           self-adversarial) + regul_rate * regularization, one launch + one fixed-order
           reduction (OpenKE strategy/NegativeSampling.py:23-32, MarginLoss.py:24-28,
           TransE.py:92-102; repo module/NegativeSampling.py:204-229).
backward = d(loss)/d(embedding tables) into dense gradient tables: for every model one wave per
           table row sums the row's contributions in batch order (no float atomics,
           bit-reproducible). With `optimizer` (an mmre.optim.SGD doing plain SGD on the tables)
           the same pass also applies its step, p <- fma(-lr, g, p) -- torch's SGD arithmetic,
           so the parameters are bit-identical to backward() + step() -- and step() then skips
           those tables (mmre_ns_fused_grad_sgd: the optimizer's re-read of the tables and the
           gradients is gone).
"""
from __future__ import annotations

import torch

from ._lib import call, lib, mark_written, ptr, require_cuda, stream_ptr

MODEL_IDS = {"transe": 0, "transe_l2": 1, "distmult": 2, "complex": 3, "rotate": 4}


class NSSpec:
    """Static description of how rows are scored (the model's forward in 'normal' mode)."""

    def __init__(self, model: str, dim: int, norm_flag: bool = False, model_margin: float | None = None,
                 phase_denom: float = 0.0):
        self.model = model
        self.model_id = MODEL_IDS[model]
        self.dim = int(dim)
        self.norm_flag = bool(norm_flag)
        self.use_model_margin = model_margin is not None
        self.model_margin = float(model_margin or 0.0)
        self.phase_denom = float(phase_denom)


def _scalar_args(spec, batch, neg, loss_margin, adv_t, regul_rate):
    return (spec.model_id, int(spec.norm_flag), spec.model_margin, int(spec.use_model_margin))


class _FusedNS(torch.autograd.Function):
    """Training (the tables need gradients): mmre_ns_fused_forward in the forward (loss,
    scores, and the gradient's slot contributions kept in the workspace), mmre_ns_fused_grad
    in the backward (every row of the gradient tables written, scaled by the upstream
    gradient; a row-owner pass with no float atomics). Otherwise mmre_ns_forward, with
    mmre_ns_backward (slots + row owner, no float atomics either) as the backward."""

    @staticmethod
    def forward(ctx, ent, rel, ent_im, rel_im, h, t, r, spec, batch, neg, loss_margin, adv_t, regul_rate, events,
                sgd):
        dev = ent.device
        N = batch * (1 + neg)
        score = torch.empty(N, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        ctx.mark_non_differentiable(score)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the (non-differentiable) scores
        ctx.fused = any(ctx.needs_input_grad[:4])
        ctx.has_im = ent_im is not None
        ctx.cfg = (spec, batch, neg, loss_margin, adv_t, regul_rate)
        ctx.sgd = sgd if ctx.fused else None
        if ctx.fused:
            E, R = int(ent.shape[0]), int(rel.shape[0])
            work = torch.empty(int(lib().mmre_ns_fused_workspace(spec.model_id, int(spec.norm_flag), batch, neg, E, R,
                                                                 spec.dim)), dtype=torch.float32, device=dev)
            if events is not None:
                events[0].record()
            call("mmre_ns_fused_forward", spec.model_id, int(spec.norm_flag), spec.model_margin,
                 int(spec.use_model_margin), ptr(ent), ptr(ent_im), ptr(rel), ptr(rel_im), E, R, spec.dim,
                 spec.phase_denom, ptr(h), ptr(t), ptr(r), batch, neg, float(loss_margin), float(adv_t),
                 float(regul_rate), ptr(score), ptr(loss), ptr(work), stream_ptr(dev))
            if events is not None:
                events[1].record()
            ctx.work = work
            ctx.events = events
        else:
            work = torch.empty(int(lib().mmre_ns_workspace(batch, neg)), dtype=torch.float32, device=dev)
            call("mmre_ns_forward", spec.model_id, int(spec.norm_flag), spec.model_margin,
                 int(spec.use_model_margin), ptr(ent), ptr(ent_im), ptr(rel), ptr(rel_im), spec.dim,
                 spec.phase_denom, ptr(h), ptr(t), ptr(r), batch, neg, float(loss_margin), float(adv_t),
                 float(regul_rate), ptr(score), ptr(loss), ptr(work), stream_ptr(dev))
        ctx.save_for_backward(ent, rel, ent_im if ent_im is not None else ent, rel_im if rel_im is not None else rel,
                              h, t, r, score)
        return loss[0], score

    @staticmethod
    def backward(ctx, g_loss, g_score):
        if g_loss is None:
            return (None,) * 15
        ent, rel, ent_im, rel_im, h, t, r, score = ctx.saved_tensors
        spec, batch, neg, loss_margin, adv_t, regul_rate = ctx.cfg
        if not ctx.has_im:
            ent_im = rel_im = None
        dev = ent.device
        gl = g_loss.reshape(1).to(torch.float32).contiguous()
        if ctx.fused:  # every row written by the call: no fills
            ge, gr = torch.empty_like(ent), torch.empty_like(rel)
            gei = torch.empty_like(ent_im) if ent_im is not None else None
            gri = torch.empty_like(rel_im) if rel_im is not None else None
            ev = ctx.events
            if ev is not None and len(ev) > 2:
                ev[2].record()
            args = (spec.model_id, int(spec.norm_flag), spec.model_margin, int(spec.use_model_margin), ptr(ent),
                    ptr(ent_im), ptr(rel), ptr(rel_im), int(ent.shape[0]), int(rel.shape[0]), spec.dim,
                    spec.phase_denom, ptr(h), ptr(t), ptr(r), batch, neg, float(loss_margin), float(adv_t),
                    float(regul_rate), ptr(score), ptr(gl), ptr(ge), ptr(gei), ptr(gr), ptr(gri), ptr(ctx.work))
            if ctx.sgd is not None:  # the optimizer's plain SGD step in the same pass (step() skips these tables)
                opt, lr, tables = ctx.sgd
                call("mmre_ns_fused_grad_sgd", *args, float(lr), stream_ptr(dev))
                mark_written(*tables)  # the SGD update rewrote the parameters in place
                opt._fused_applied(tables)
            else:
                call("mmre_ns_fused_grad", *args, stream_ptr(dev))
            if ev is not None and len(ev) > 2:
                ev[3].record()
            ctx.work = ctx.events = ctx.sgd = None
            return ge, gr, gei, gri, None, None, None, None, None, None, None, None, None, None, None
        # deterministic rows backward (slots + row owner): writes every row, no fills
        E, R = int(ent.shape[0]), int(rel.shape[0])
        ge, gr = torch.empty_like(ent), torch.empty_like(rel)
        gei = torch.empty_like(ent_im) if ent_im is not None else None
        gri = torch.empty_like(rel_im) if rel_im is not None else None
        nw = int(lib().mmre_rows_backward_workspace(spec.model_id, batch * (1 + neg), E, R, spec.dim))
        work = torch.empty(nw, dtype=torch.float32, device=dev)
        call("mmre_ns_backward", spec.model_id, int(spec.norm_flag), spec.model_margin, int(spec.use_model_margin),
             ptr(ent), ptr(ent_im), ptr(rel), ptr(rel_im), spec.dim, spec.phase_denom, ptr(h), ptr(t), ptr(r),
             batch, neg, float(loss_margin), float(adv_t), float(regul_rate), ptr(score), ptr(gl), ptr(ge), ptr(gei),
             ptr(gr), ptr(gri), E, R, ptr(work), nw, stream_ptr(dev))
        return ge, gr, gei, gri, None, None, None, None, None, None, None, None, None, None, None


def fused_ns_loss(spec: NSSpec, ent, rel, h, t, r, batch: int, neg: int, loss_margin: float,
                  adv_temperature: float | None = None, regul_rate: float = 0.0, ent_im=None, rel_im=None,
                  events=None, optimizer=None):
    """Returns (loss scalar tensor, scores (B*(1+k),)). Differentiable w.r.t. the tables.
    events: optional torch.cuda.Events recorded around the C-ABI calls alone (training mode), for
    kernel timing: (start, end) of mmre_ns_fused_forward, and with four, (start, end) of the
    backward's mmre_ns_fused_grad.
    optimizer: an mmre.optim.SGD over the tables; when its step is plain SGD and the tables have
    no gradient yet (zero_grad(set_to_none=True): autograd will assign, not accumulate), the
    backward applies the step as well (mmre_ns_fused_grad_sgd) and optimizer.step() skips the
    tables. The parameters afterwards are bit-identical to backward() + step(); p.grad is still
    written. Otherwise the optimizer is ignored here."""
    require_cuda(ent, rel, h, t, r, ent_im, rel_im)
    h, t, r = (x.to(torch.int64).contiguous() for x in (h, t, r))
    if ent.dtype != torch.float32 or rel.dtype != torch.float32:
        raise TypeError("fused_ns_loss: float32 tables")
    tables = [x for x in (ent, rel, ent_im, rel_im) if x is not None]
    sgd = None
    if optimizer is not None and hasattr(optimizer, "fusable_lr"):
        lr = optimizer.fusable_lr(tables)
        if lr is not None:
            sgd = (optimizer, lr, tables)
    return _FusedNS.apply(ent.contiguous(), rel.contiguous(), None if ent_im is None else ent_im.contiguous(),
                          None if rel_im is None else rel_im.contiguous(), h, t, r, spec, int(batch), int(neg),
                          float(loss_margin), float(adv_temperature or 0.0), float(regul_rate), events, sgd)


class _ScoreRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ent, rel, ent_im, rel_im, h, t, r, spec):
        n = int(h.shape[0])
        dev = ent.device
        score = torch.empty(n, dtype=torch.float32, device=dev)
        work = torch.empty(int(lib().mmre_ns_workspace(n, 0)), dtype=torch.float32, device=dev)
        call("mmre_ns_forward", spec.model_id, int(spec.norm_flag), spec.model_margin, int(spec.use_model_margin),
             ptr(ent), ptr(ent_im), ptr(rel), ptr(rel_im), spec.dim, spec.phase_denom, ptr(h), ptr(t), ptr(r), n, 0,
             0.0, 0.0, 0.0, ptr(score), None, ptr(work), stream_ptr(dev))
        ctx.save_for_backward(ent, rel, ent_im if ent_im is not None else ent, rel_im if rel_im is not None else rel,
                              h, t, r)
        ctx.has_im = ent_im is not None
        ctx.spec = spec
        return score

    @staticmethod
    def backward(ctx, g_score):
        ent, rel, ent_im, rel_im, h, t, r = ctx.saved_tensors
        spec = ctx.spec
        if not ctx.has_im:
            ent_im = rel_im = None
        g = g_score.to(torch.float32).contiguous()
        # deterministic rows backward (slots + row owner, no float atomics): writes every row
        E, R = int(ent.shape[0]), int(rel.shape[0])
        ge, gr = torch.empty_like(ent), torch.empty_like(rel)
        gei = torch.empty_like(ent_im) if ent_im is not None else None
        gri = torch.empty_like(rel_im) if rel_im is not None else None
        n = int(h.shape[0])
        nw = int(lib().mmre_rows_backward_workspace(spec.model_id, n, E, R, spec.dim))
        work = torch.empty(nw, dtype=torch.float32, device=ent.device)
        call("mmre_score_rows_backward", spec.model_id, int(spec.norm_flag), spec.model_margin,
             int(spec.use_model_margin), ptr(ent), ptr(ent_im), ptr(rel), ptr(rel_im), spec.dim, spec.phase_denom,
             ptr(h), ptr(t), ptr(r), n, ptr(g), ptr(ge), ptr(gei), ptr(gr), ptr(gri), E, R, ptr(work), nw,
             stream_ptr(ent.device))
        return ge, gr, gei, gri, None, None, None, None


def score_rows(spec: NSSpec, ent, rel, h, t, r, ent_im=None, rel_im=None):
    """model(data) in 'normal' mode for arbitrary rows (differentiable w.r.t. the tables)."""
    require_cuda(ent, rel, h, t, r, ent_im, rel_im)
    h, t, r = (x.to(torch.int64).contiguous() for x in (h, t, r))
    c = lambda x: None if x is None else x.contiguous()
    return _ScoreRows.apply(c(ent), c(rel), c(ent_im), c(rel_im), h, t, r, spec)


class OpenKETrainStep:
    """One OpenKE training step for TransE -- Trainer.train_one_step (Trainer.py:43-54) over the
    loader's Base.cpp sampling, strategy/NegativeSampling + MarginLoss, optim.SGD -- as ONE C-ABI
    call: the values of sampler.sample(B, neg, 0, mode) + fused_ns_loss(...).backward() +
    SGD.step(), bit for bit (tests/test_ns_full_gpu.py). The parameters are updated in place;
    ent.grad / rel.grad hold the step's gradient tables, `batch` the batch the step trained on,
    `score` the row scores. Calling it returns the loss tensor (device).

    pipeline=True (default; mmre_ns_step_openke_pipe): like a prefetching data loader, each step
    also draws the NEXT batch (in its gradient launch, beside the row owner) and writes the
    norms of the rows it updates, so the next step is two launches (the fused loss kernel, the
    row owner) instead of three. Batches, losses, gradients and parameters are the unpipelined
    sequence's; the sampler is one batch ahead between calls (as with any prefetching loader,
    another consumer drawing from the same sampler between steps sees batch i + 2, and the
    prefetched batch is then discarded). The prefetch is used only while it is current: ent /
    rel modified in place since the previous call (torch's version counters) re-run the
    pre-pass; the sampler drawn from or reseeded elsewhere re-draws the batch.
    pipeline=False: mmre_ns_step_openke (three launches every step).

    DistMult / ComplEx / RotatE (mmre_ns_step_openke_gen_pipe; ent_im / rel_im for ComplEx, the
    spec's model margin and phase for RotatE): the generic fused path's kernels -- forward,
    slot records, row owner with SGD -- with the loss reduction and (pipeline=True) the next
    batch's sampler in the row owner's grid: three launches a step instead of the drop-in
    path's five (sampler, forward, loss reduction, slots, row owner), the same values."""

    GENERIC = ("distmult", "complex", "rotate")

    def __init__(self, sampler, spec: NSSpec, ent, rel, batch: int, neg: int, loss_margin: float, lr: float,
                 adv_temperature: float | None = None, regul_rate: float = 0.0, mode: int = 0,
                 pipeline: bool = True, ent_im=None, rel_im=None):
        self.generic = spec.model in self.GENERIC
        if not self.generic and (spec.model not in ("transe", "transe_l2") or spec.use_model_margin):
            raise ValueError("OpenKETrainStep: TransE without a model margin, DistMult, ComplEx or RotatE")
        if (spec.model == "complex") != (ent_im is not None and rel_im is not None):
            raise ValueError("OpenKETrainStep: ComplEx takes ent_im and rel_im (and only ComplEx)")
        require_cuda(ent, rel, ent_im, rel_im)
        dev = ent.device
        self.ent_im, self.rel_im = ent_im, rel_im
        self.sampler, self.spec, self.ent, self.rel = sampler, spec, ent, rel
        self.B, self.K, self.mode = int(batch), int(neg), int(mode)
        self.margin, self.lr = float(loss_margin), float(lr)
        self.adv, self.regul = float(adv_temperature or 0.0), float(regul_rate)
        self.pipeline = bool(pipeline)
        E, R = int(ent.shape[0]), int(rel.shape[0])
        n = self.B * (1 + self.K)
        self.work = torch.empty(int(lib().mmre_ns_fused_workspace(spec.model_id, int(spec.norm_flag), self.B, self.K, E,
                                                                  R, spec.dim)), dtype=torch.float32, device=dev)
        self.score = torch.empty(n, dtype=torch.float32, device=dev)
        self.loss = torch.empty(1, dtype=torch.float32, device=dev)
        mk = lambda: dict(batch_h=torch.empty(n, dtype=torch.int64, device=dev),
                          batch_t=torch.empty(n, dtype=torch.int64, device=dev),
                          batch_r=torch.empty(n, dtype=torch.int64, device=dev),
                          batch_y=torch.empty(n, dtype=torch.float32, device=dev))
        self._bufs = [mk(), mk()] if self.pipeline else [mk()]
        self.batch = self._bufs[0]
        self._parity = 0
        self._ready = None  # (sampler draws, (ent, rel) versions) right after a call that prefetched
        self.ge, self.gr = torch.empty_like(ent), torch.empty_like(rel)  # the step's gradient tables
        self.gei = torch.empty_like(ent_im) if ent_im is not None else None
        self.gri = torch.empty_like(rel_im) if rel_im is not None else None

    def invalidate(self):
        """Forget the prefetch -- after replaying captured graphs of this step, whose launches this
        object's host state does not follow: the next call draws a batch and runs the pre-pass."""
        self._ready = None

    def _state(self):
        return (self.sampler.draws, tuple(t._version for t in (self.ent, self.rel, self.ent_im, self.rel_im)
                                          if t is not None))

    def _generic_call(self, prefetch: bool):
        s = self.spec
        E, R = int(self.ent.shape[0]), int(self.rel.shape[0])
        p = self._parity
        cur = self._bufs[p]
        nxt = self._bufs[1 - p] if (self.pipeline and prefetch) else None
        st = self._state()
        prepared = 1 if (self.pipeline and self._ready is not None and self._ready[0] == st[0]) else 0
        args = self.sampler.step_args(self.B, self.K, self.mode, cur, advance=not prepared)
        call("mmre_ns_step_openke_gen_pipe", *args, s.model_id, s.model_margin, int(s.use_model_margin), ptr(self.ent),
             ptr(self.ent_im), ptr(self.rel), ptr(self.rel_im), E, R, s.dim, s.phase_denom, self.B, self.K,
             self.margin, self.adv, self.regul, ptr(self.score), ptr(self.loss), ptr(self.ge), ptr(self.gei),
             ptr(self.gr), ptr(self.gri), ptr(self.work), self.lr, stream_ptr(self.ent.device), prepared,
             ptr(nxt["batch_h"]) if nxt else None, ptr(nxt["batch_t"]) if nxt else None,
             ptr(nxt["batch_r"]) if nxt else None, ptr(nxt["batch_y"]) if nxt else None)
        mark_written(self.ent, self.rel, self.ent_im, self.rel_im)
        self.batch = cur
        if nxt is not None:
            self.sampler.advance(self.B, self.K, self.mode)
            self._parity = 1 - p
            self._ready = self._state()
        else:
            self._ready = None
        self.ent.grad, self.rel.grad = self.ge, self.gr
        if self.ent_im is not None:
            self.ent_im.grad, self.rel_im.grad = self.gei, self.gri
        return self.loss[0]

    def __call__(self, prefetch: bool = True):
        """One training step. prefetch=False (pipeline=True): do not draw the next batch -- the
        last step of a run, leaving the sampler exactly where the unpipelined sequence does."""
        if self.generic:
            return self._generic_call(prefetch)
        s = self.spec
        E, R = int(self.ent.shape[0]), int(self.rel.shape[0])
        tail = (s.model_id, int(s.norm_flag), ptr(self.ent), ptr(self.rel), E, R, s.dim, self.B, self.K, self.margin,
                self.adv, self.regul, ptr(self.score), ptr(self.loss), ptr(self.ge), ptr(self.gr), ptr(self.work),
                self.lr, stream_ptr(self.ent.device))
        if not self.pipeline:
            call("mmre_ns_step_openke", *self.sampler.step_args(self.B, self.K, self.mode, self.batch), *tail)
            mark_written(self.ent, self.rel)
        else:
            p = self._parity
            cur, nxt = self._bufs[p], (self._bufs[1 - p] if prefetch else None)
            st = self._state()
            # bit 0: the current batch was drawn by the previous call's gradient launch (else this
            # call's first launch draws it); bit 1: the pre-pass that launch made is current
            prepared = 0
            if self._ready is not None:
                prepared = (1 if self._ready[0] == st[0] else 0) | (2 if self._ready[1] == st[1] else 0)
            args = self.sampler.step_args(self.B, self.K, self.mode, cur, advance=not prepared & 1)
            nx = (ptr(nxt["batch_h"]), ptr(nxt["batch_t"]), ptr(nxt["batch_r"]), ptr(nxt["batch_y"])) if nxt \
                else (None, None, None, None)
            call("mmre_ns_step_openke_pipe", *args, *tail, prepared, p, *nx)
            mark_written(self.ent, self.rel)  # the SGD update, before the prefetch's state is recorded
            self.batch = cur
            if nxt is not None:
                self.sampler.advance(self.B, self.K, self.mode)
                self._parity = 1 - p
                self._ready = self._state()
            else:
                self._ready = None
        self.ent.grad, self.rel.grad = self.ge, self.gr  # as backward() leaves them
        return self.loss[0]
