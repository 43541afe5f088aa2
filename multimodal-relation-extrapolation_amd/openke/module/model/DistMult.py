"""DistMult (OpenKE/openke/module/model/DistMult.py:5-72) on libmmre_hip.so."""
import torch
import torch.nn as nn

from mmre.link import ScoreSpec
from mmre.ns import NSSpec

from .Model import Model


class DistMult(Model):
    def __init__(self, ent_tot, rel_tot, dim=100, margin=None, epsilon=None):
        super().__init__(ent_tot, rel_tot)
        self.dim = dim
        self.margin = margin
        self.epsilon = epsilon
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

    def _tables(self):
        return self.ent_embeddings.weight, self.rel_embeddings.weight, None, None

    def ns_spec(self):
        return NSSpec("distmult", self.dim)

    def score_spec(self):
        return ScoreSpec(model="distmult", ent=self.ent_embeddings.weight, rel=self.rel_embeddings.weight,
                         dim=self.dim, pred_kind=2)

    def _predict_transform(self, score):
        return -score

    def l3_regularization(self):
        return self.ent_embeddings.weight.norm(p=3) ** 3 + self.rel_embeddings.weight.norm(p=3) ** 3
