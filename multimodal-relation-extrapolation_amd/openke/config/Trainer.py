"""Trainer (OpenKE/openke/config/Trainer.py:16-134): same constructor, setters and run() loop.
Batches arrive from the GPU sampler already on the device; the strategy's forward/backward is
the fused HIP loss; the optimizer step is torch's."""
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
        if hasattr(self.model, "fuse_optimizer") and hasattr(self.optimizer, "fusable_lr"):
            # the fused negative-sampling backward applies the plain SGD step itself (bit-identical)
            self.model.fuse_optimizer(self.optimizer)
        for epoch in range(self.train_times):
            res = 0.0
            for data in self.data_loader:
                res += self.train_one_step(data)
            self.log.append(res)
            if self.save_steps and self.checkpoint_dir and (epoch + 1) % self.save_steps == 0:
                self.model.save_checkpoint(os.path.join(self.checkpoint_dir + "-" + str(epoch) + ".ckpt"))

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
