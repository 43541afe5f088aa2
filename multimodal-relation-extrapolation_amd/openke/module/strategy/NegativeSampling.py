"""NegativeSampling strategy (OpenKE/openke/module/strategy/NegativeSampling.py:3-32).

With a MarginLoss and 'normal'-mode batches the forward is ONE fused HIP launch sequence
(mmre.ns.fused_ns_loss): row scores -> positive/negative split -> (self-adversarial) hinge ->
mean -> + regul_rate * regularization, with a fused backward into the embedding tables.
Other losses / cross-sampling modes score through model(data) (HIP) and apply the loss
module on the score tensors. `fuse_optimizer(opt)` (the Trainer calls it for its mmre.optim.SGD)
lets that backward also apply the optimizer's plain SGD step to the tables in the same pass
(bit-identical parameters; step() then skips them)."""
from mmre.ns import fused_ns_loss

from ..loss.MarginLoss import MarginLoss
from .Strategy import Strategy


class NegativeSampling(Strategy):
    def __init__(self, model=None, loss=None, batch_size=256, regul_rate=0.0, l3_regul_rate=0.0):
        super().__init__()
        self.model = model
        self.loss = loss
        self.batch_size = batch_size
        self.regul_rate = regul_rate
        self.l3_regul_rate = l3_regul_rate
        self.fused_optimizer = None

    def fuse_optimizer(self, optimizer):
        self.fused_optimizer = optimizer

    def _get_positive_score(self, score):
        return score[:self.batch_size].view(-1, self.batch_size).permute(1, 0)

    def _get_negative_score(self, score):
        return score[self.batch_size:].view(-1, self.batch_size).permute(1, 0)

    def forward(self, data):
        mode = data.get("mode", "normal")
        if isinstance(self.loss, MarginLoss) and mode == "normal":
            ent, rel, ent_im, rel_im = self.model._tables()
            dev = ent.device
            h = data["batch_h"].to(dev)
            t = data["batch_t"].to(dev)
            r = data["batch_r"].to(dev)
            n = int(h.shape[0])
            neg = n // self.batch_size - 1
            margin, adv = self.loss.fused_args()
            loss_res, _ = fused_ns_loss(self.model.ns_spec(), ent, rel, h, t, r, self.batch_size, neg, margin,
                                        adv, self.regul_rate, ent_im=ent_im, rel_im=rel_im,
                                        optimizer=self.fused_optimizer if self.l3_regul_rate == 0 else None)
        else:
            score = self.model(data)
            loss_res = self.loss(self._get_positive_score(score), self._get_negative_score(score))
            if self.regul_rate != 0:
                loss_res = loss_res + self.regul_rate * self.model.regularization(data)
        if self.l3_regul_rate != 0:
            loss_res = loss_res + self.l3_regul_rate * self.model.l3_regularization()
        return loss_res
