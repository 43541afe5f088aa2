"""Model base class (OpenKE/openke/module/model/Model.py:6-17) plus the two hooks the MI355X
engine uses: `score_spec()` (link-prediction sweep) and `ns_spec()` (fused training loss).

forward(data) follows OpenKE: data = {'batch_h', 'batch_t', 'batch_r': index tensors, 'mode'}.
'normal' mode scores row-wise; 'head_batch'/'tail_batch' broadcast the candidate side against
r.shape[0] queries (TransE.py:67-70) -- here both run on libmmre_hip.so (mmre.ns.score_rows).
"""
import numpy as np
import torch

from mmre import ns as _ns

from ..BaseModule import BaseModule


class Model(BaseModule):
    def __init__(self, ent_tot, rel_tot):
        super().__init__()
        self.ent_tot = ent_tot
        self.rel_tot = rel_tot

    # ---- engine hooks (overridden) ----
    def score_spec(self):
        raise NotImplementedError

    def ns_spec(self):
        raise NotImplementedError

    def _tables(self):
        """(ent, rel, ent_im, rel_im) weight tensors in the engine's layout."""
        raise NotImplementedError

    # ---- OpenKE API ----
    def _expand(self, data):
        dev = self._tables()[0].device
        h = torch.as_tensor(data["batch_h"]).to(dev).long().reshape(-1)
        t = torch.as_tensor(data["batch_t"]).to(dev).long().reshape(-1)
        r = torch.as_tensor(data["batch_r"]).to(dev).long().reshape(-1)
        mode = data.get("mode", "normal")
        if mode != "normal":
            # view(-1, r.shape[0], d): candidate i of query j at [i * n + j] (TransE.py:67-70)
            n = r.shape[0]
            m = max(h.shape[0], t.shape[0]) // n
            idx = torch.arange(m * n, device=dev)
            h = h[idx % h.shape[0]] if h.shape[0] != m * n else h
            t = t[idx % t.shape[0]] if t.shape[0] != m * n else t
            r = r[idx % n]
        return h, t, r

    def forward(self, data):
        ent, rel, ent_im, rel_im = self._tables()
        h, t, r = self._expand(data)
        return _ns.score_rows(self.ns_spec(), ent, rel, h, t, r, ent_im=ent_im, rel_im=rel_im)

    def _predict_transform(self, score):
        return score

    def predict(self, data):
        with torch.no_grad():
            score = self._predict_transform(self.forward(data))
        return score.cpu().numpy()

    def regularization(self, data):
        ent, rel, ent_im, rel_im = self._tables()
        h, t, r = self._expand(data)
        if ent_im is None:
            return (torch.mean(ent[h] ** 2) + torch.mean(ent[t] ** 2) + torch.mean(rel[r] ** 2)) / 3
        return (torch.mean(ent[h] ** 2) + torch.mean(ent_im[h] ** 2) + torch.mean(ent[t] ** 2) +
                torch.mean(ent_im[t] ** 2) + torch.mean(rel[r] ** 2) + torch.mean(rel_im[r] ** 2)) / 6
