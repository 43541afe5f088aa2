"""RotatE (OpenKE/openke/module/model/RotatE.py:6-103) on libmmre_hip.so."""
import torch
import torch.nn as nn

from mmre.link import ScoreSpec, rotate_phase_denom
from mmre.ns import NSSpec

from .Model import Model


class RotatE(Model):
    def __init__(self, ent_tot, rel_tot, dim=100, margin=6.0, epsilon=2.0):
        super().__init__(ent_tot, rel_tot)
        self.margin_value = float(margin)
        self.epsilon = epsilon
        self.dim_e = dim * 2
        self.dim_r = dim
        self.ent_embeddings = nn.Embedding(self.ent_tot, self.dim_e)
        self.rel_embeddings = nn.Embedding(self.rel_tot, self.dim_r)
        self.ent_embedding_range = nn.Parameter(torch.Tensor([(margin + epsilon) / self.dim_e]),
                                                requires_grad=False)
        nn.init.uniform_(self.ent_embeddings.weight.data, -self.ent_embedding_range.item(),
                         self.ent_embedding_range.item())
        self.rel_embedding_range = nn.Parameter(torch.Tensor([(margin + epsilon) / self.dim_r]),
                                                requires_grad=False)
        nn.init.uniform_(self.rel_embeddings.weight.data, -self.rel_embedding_range.item(),
                         self.rel_embedding_range.item())
        self.margin = nn.Parameter(torch.Tensor([margin]), requires_grad=False)

    def _denom(self):
        return rotate_phase_denom(self.margin_value, self.epsilon, self.dim_r)

    def _tables(self):
        return self.ent_embeddings.weight, self.rel_embeddings.weight, None, None

    def ns_spec(self):
        return NSSpec("rotate", self.dim_r, model_margin=float(self.margin.item()), phase_denom=self._denom())

    def score_spec(self):
        # predict = -forward = -(m - s)   (RotatE.py:86-91)
        return ScoreSpec(model="rotate", ent=self.ent_embeddings.weight, rel=self.rel_embeddings.weight,
                         dim=self.dim_r, pred_kind=3, margin=float(self.margin.item()), phase_denom=self._denom())

    def _predict_transform(self, score):
        return -score
