"""MarginLoss (OpenKE/openke/module/loss/MarginLoss.py:8-33).

Inside strategy.NegativeSampling the whole score -> hinge -> mean (+ regularization) graph runs
as one fused HIP kernel (mmre.ns); called standalone on (p, n) score tensors it evaluates the
same formula with device tensor ops."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .Loss import Loss


class MarginLoss(Loss):
    def __init__(self, adv_temperature=None, margin=6.0):
        super().__init__()
        self.margin = nn.Parameter(torch.Tensor([margin]), requires_grad=False)
        if adv_temperature is not None:
            self.adv_temperature = nn.Parameter(torch.Tensor([adv_temperature]), requires_grad=False)
            self.adv_flag = True
        else:
            self.adv_flag = False

    def get_weights(self, n_score):
        return F.softmax(-n_score * self.adv_temperature, dim=-1).detach()

    def forward(self, p_score, n_score):
        m = self.margin.to(p_score.device)
        if self.adv_flag:
            return (self.get_weights(n_score) * torch.max(p_score - n_score, -m)).sum(dim=-1).mean() + m
        return (torch.max(p_score - n_score, -m)).mean() + m

    def predict(self, p_score, n_score):
        return self.forward(p_score, n_score).cpu().data.numpy()

    # fused-kernel parameters
    def fused_args(self):
        return float(self.margin.item()), (float(self.adv_temperature.item()) if self.adv_flag else None)
