"""TransE (OpenKE/openke/module/model/TransE.py:6-110) on libmmre_hip.so."""
import torch
import torch.nn as nn

from mmre.link import ScoreSpec
from mmre.ns import NSSpec

from .Model import Model


class TransE(Model):
    def __init__(self, ent_tot, rel_tot, dim=100, p_norm=1, norm_flag=True, margin=None, epsilon=None):
        super().__init__(ent_tot, rel_tot)
        if p_norm not in (1, 2):
            raise ValueError("TransE: p_norm must be 1 or 2")
        self.dim = dim
        self.margin = margin
        self.epsilon = epsilon
        self.norm_flag = norm_flag
        self.p_norm = p_norm
        self.ent_embeddings = nn.Embedding(self.ent_tot, self.dim)
        self.rel_embeddings = nn.Embedding(self.rel_tot, self.dim)
        if margin is None or epsilon is None:
            nn.init.xavier_uniform_(self.ent_embeddings.weight.data)
            nn.init.xavier_uniform_(self.rel_embeddings.weight.data)
        else:
            self.embedding_range = nn.Parameter(torch.Tensor([(self.margin + self.epsilon) / self.dim]),
                                                requires_grad=False)
            nn.init.uniform_(self.ent_embeddings.weight.data, -self.embedding_range.item(),
                             self.embedding_range.item())
            nn.init.uniform_(self.rel_embeddings.weight.data, -self.embedding_range.item(),
                             self.embedding_range.item())
        if margin is not None:
            self.margin = nn.Parameter(torch.Tensor([margin]), requires_grad=False)
            self.margin_flag = True
        else:
            self.margin_flag = False

    def _m(self):
        return float(self.margin.item()) if self.margin_flag else None

    def _tables(self):
        return self.ent_embeddings.weight, self.rel_embeddings.weight, None, None

    def ns_spec(self):
        return NSSpec("transe" if self.p_norm == 1 else "transe_l2", self.dim, norm_flag=self.norm_flag,
                      model_margin=self._m())

    def score_spec(self):
        # predict() = margin - forward = m - (m - s) when margin_flag, else s   (TransE.py:104-110)
        return ScoreSpec(model="transe" if self.p_norm == 1 else "transe_l2", ent=self.ent_embeddings.weight,
                         rel=self.rel_embeddings.weight, dim=self.dim, norm_flag=self.norm_flag,
                         pred_kind=1 if self.margin_flag else 0, margin=self._m() or 0.0)

    def _predict_transform(self, score):
        return self.margin - score if self.margin_flag else score
