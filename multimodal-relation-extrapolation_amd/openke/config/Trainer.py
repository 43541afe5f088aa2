"""Trainer (OpenKE/openke/config/Trainer.py:16-134): same constructor, setters and run() loop.
Batches arrive from the GPU sampler already on the device; the strategy's forward/backward is
the fused HIP loss; plain SGD runs inside the fused backward (mmre.optim.SGD). For TransE +
MarginLoss + SGD with 'normal' sampling (TransE, DistMult, ComplEx, RotatE), run() takes the
whole step as one C-ABI call (mmre.ns.OpenKETrainStep: same batches, losses and parameters, bit
for bit)."""
import os

import numpy as np
import torch
import torch.optim as optim


class Trainer(object):
    def __init__(self, model=None, data_loader=None, train_times=1000, alpha=0.5, use_gpu=True, opt_method="sgd",
                 save_steps=None, checkpoint_dir=None):
        self.work_threads = 8
        self.train_times = train_times
        self.opt_method = opt_method
        self.optimizer = None
        self.lr_decay = 0
        self.weight_decay = 0
        self.alpha = alpha
        self.model = model
        self.data_loader = data_loader
        self.use_gpu = use_gpu
        self.save_steps = save_steps
        self.checkpoint_dir = checkpoint_dir
        self.log = []
        # run() takes the one-call TransE step (mmre_ns_step_openke) when the configuration allows
        # it -- same values as train_one_step, bit for bit (tests/test_api_gpu.py); False forces the
        # per-batch path
        self.one_call_step = True

    def to_var(self, x, use_gpu):
        if isinstance(x, torch.Tensor):
            return x.cuda() if use_gpu and not x.is_cuda else x
        t = torch.from_numpy(np.asarray(x))
        return t.cuda() if use_gpu else t

    def train_one_step(self, data):
        self.optimizer.zero_grad()
        loss = self.model({
            "batch_h": self.to_var(data["batch_h"], self.use_gpu),
            "batch_t": self.to_var(data["batch_t"], self.use_gpu),
            "batch_r": self.to_var(data["batch_r"], self.use_gpu),
            "batch_y": self.to_var(data["batch_y"], self.use_gpu),
            "mode": data["mode"],
        })
        loss.backward()
        self.optimizer.step()
        return loss.item()

    def make_optimizer(self):
        p = self.model.parameters()
        m = (self.opt_method or "sgd").lower()
        if m == "adagrad":
            return optim.Adagrad(p, lr=self.alpha, lr_decay=self.lr_decay, weight_decay=self.weight_decay)
        if m == "adadelta":
            return optim.Adadelta(p, lr=self.alpha, weight_decay=self.weight_decay)
        if m == "adam":
            return optim.Adam(p, lr=self.alpha, weight_decay=self.weight_decay)
        from mmre.optim import SGD  # plain SGD: one HIP launch over the tables (torch's step otherwise)
        return SGD(p, lr=self.alpha, weight_decay=self.weight_decay)

    def run(self):
        if self.use_gpu:
            self.model.cuda()
        if self.optimizer is None:
            self.optimizer = self.make_optimizer()
        fusing = hasattr(self.model, "fuse_optimizer") and hasattr(self.optimizer, "fusable_lr")
        if fusing:
            # the fused negative-sampling backward applies the plain SGD step itself (bit-identical);
            # only for the duration of this run (train_one_step: zero_grad, ONE backward, step)
            self.model.fuse_optimizer(self.optimizer)
        try:
            self._run_epochs()
        finally:
            if fusing:
                self.model.fuse_optimizer(None)

    def _run_epochs(self):
        fast = self._one_call_step() if self.one_call_step else None
        self.used_one_call_step = fast is not None
        for epoch in range(self.train_times):
            res = 0.0
            if fast is not None:
                step, group = fast
                nb = len(self.data_loader)
                for b in range(nb):
                    step.lr = float(group["lr"])
                    # the step draws the next batch beside its gradient (a prefetching loader),
                    # except after the run's last batch: the sampler ends where the per-batch path does
                    res += float(step(prefetch=not (epoch == self.train_times - 1 and b == nb - 1)).item())
            else:
                for data in self.data_loader:
                    res += self.train_one_step(data)
            self.log.append(res)
            if self.save_steps and self.checkpoint_dir and (epoch + 1) % self.save_steps == 0:
                self.model.save_checkpoint(os.path.join(self.checkpoint_dir + "-" + str(epoch) + ".ckpt"))

    def _one_call_step(self):
        """(mmre.ns.OpenKETrainStep, its optimizer group) when the whole step -- the loader's
        Base.cpp sampling, NegativeSampling + MarginLoss on TransE, DistMult, ComplEx or RotatE,
        plain SGD -- can run as one C-ABI call (mmre_ns_step_openke_pipe for TransE,
        mmre_ns_step_openke_gen_pipe for the others); else None (train_one_step)."""
        try:
            from ..data.TrainDataLoader import TrainDataLoader
            from ..module.loss.MarginLoss import MarginLoss
            from ..module.strategy.NegativeSampling import NegativeSampling
            from mmre.ns import OpenKETrainStep
        except ImportError:
            return None
        m, dl = self.model, self.data_loader
        if not (isinstance(m, NegativeSampling) and isinstance(m.loss, MarginLoss) and isinstance(dl, TrainDataLoader)):
            return None
        if m.l3_regul_rate != 0 or dl.sampling_mode != "normal" or dl.negative_rel != 0 or m.batch_size != dl.batch_size:
            return None
        if not (hasattr(m.model, "ns_spec") and hasattr(m.model, "_tables")):
            return None
        spec = m.model.ns_spec()
        ent, rel, ent_im, rel_im = m.model._tables()
        generic = spec.model in OpenKETrainStep.GENERIC
        if generic:
            # DistMult / ComplEx / RotatE: mmre_ns_step_openke_gen_pipe (the generic kernels' shapes)
            if (spec.model == "complex") != (ent_im is not None and rel_im is not None):
                return None
            if spec.dim > 512 or dl.negative_ent > 512 or dl.negative_ent < 1:
                return None
        else:
            if spec.model not in ("transe", "transe_l2") or spec.use_model_margin or ent_im is not None:
                return None
            if spec.dim > 512 or dl.negative_ent > 32 or dl.negative_ent < 1:  # the fused kernel's shapes
                return None
        tables = [x for x in (ent, rel, ent_im, rel_im) if x is not None]
        if not hasattr(self.optimizer, "fusable_lr") or self.optimizer.fusable_lr(tables) is None:
            return None
        group = next(g for g in self.optimizer.param_groups if any(p is ent for p in g["params"]))
        margin, adv = m.loss.fused_args()
        step = OpenKETrainStep(dl.sampler, spec, ent, rel, dl.batch_size, dl.negative_ent, margin, float(group["lr"]),
                               adv_temperature=adv, regul_rate=m.regul_rate, ent_im=ent_im, rel_im=rel_im)
        return step, group

    def set_model(self, model):
        self.model = model

    def set_use_gpu(self, use_gpu):
        self.use_gpu = use_gpu

    def set_alpha(self, alpha):
        self.alpha = alpha

    def set_lr_decay(self, lr_decay):
        self.lr_decay = lr_decay

    def set_weight_decay(self, weight_decay):
        self.weight_decay = weight_decay

    def set_opt_method(self, opt_method):
        self.opt_method = opt_method

    def set_train_times(self, train_times):
        self.train_times = train_times

    def set_save_steps(self, save_steps, checkpoint_dir=None):
        self.save_steps = save_steps
        if not self.checkpoint_dir:
            self.set_checkpoint_dir(checkpoint_dir)

    def set_checkpoint_dir(self, checkpoint_dir):
        self.checkpoint_dir = checkpoint_dir
