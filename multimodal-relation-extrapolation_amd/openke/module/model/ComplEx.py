"""ComplEx (OpenKE/openke/module/model/ComplEx.py:5-62) on libmmre_hip.so."""
import torch.nn as nn

from mmre.link import ScoreSpec
from mmre.ns import NSSpec

from .Model import Model


class ComplEx(Model):
    def __init__(self, ent_tot, rel_tot, dim=100):
        super().__init__(ent_tot, rel_tot)
        self.dim = dim
        self.ent_re_embeddings = nn.Embedding(self.ent_tot, self.dim)
        self.ent_im_embeddings = nn.Embedding(self.ent_tot, self.dim)
        self.rel_re_embeddings = nn.Embedding(self.rel_tot, self.dim)
        self.rel_im_embeddings = nn.Embedding(self.rel_tot, self.dim)
        for e in (self.ent_re_embeddings, self.ent_im_embeddings, self.rel_re_embeddings, self.rel_im_embeddings):
            nn.init.xavier_uniform_(e.weight.data)

    def _tables(self):
        return (self.ent_re_embeddings.weight, self.rel_re_embeddings.weight, self.ent_im_embeddings.weight,
                self.rel_im_embeddings.weight)

    def ns_spec(self):
        return NSSpec("complex", self.dim)

    def score_spec(self):
        return ScoreSpec(model="complex", ent=self.ent_re_embeddings.weight, rel=self.rel_re_embeddings.weight,
                         ent_im=self.ent_im_embeddings.weight, rel_im=self.rel_im_embeddings.weight, dim=self.dim,
                         pred_kind=2)

    def _predict_transform(self, score):
        return -score
