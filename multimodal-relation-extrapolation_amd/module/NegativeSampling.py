"""Repo-level NegativeSampling strategy (module/NegativeSampling.py:19-375) on libmmre_hip.so.

forward(local_global_id, edge_index, edge_type, batch) keeps the reference contract:
    x_gcn, rel_emb, batch_output = self.model(edge_index, edge_type, batch, deterministic)
    -> GPU filtered negative sampler (RepoSampler)        (neg_sample_fn, :114-140)
    -> fused TransE/DistMult score + MarginLoss + 0.5 * regularization (one HIP launch pair)
    -> loss = loss_image_text + gcn_w * loss_res_gcn + contrastive_w * contrastive_loss  (:271-276)
including the reference's in-place aliasing (struct_loss += regul mutates loss_res_gcn, so the
returned gcn_loss IS struct_loss and the total carries gcn_w * regul_rate * regul; P9).
The multimodal reconstruction losses (image/text, :231-269) come from the upstream encoder: pass
them in batch_output as 'image_loss' / 'text_loss' (scalars) when present."""
import numpy as np
import torch
import torch.nn as nn

from mmre.ns import NSSpec, fused_ns_loss, score_rows
from mmre.sampler import RepoSampler

from .submodule import BaseModule


class NegativeSampling(BaseModule):
    def __init__(self, args, whole_triples, model=None, loss_fn=None, regul_rate=0.5, neg_ent=1,
                 sampling_mode="normal", bern_flag=False, filter_flag=True, score_norm_flag=False, seed=0):
        super().__init__()
        self.args = args
        self.model = model
        self.loss_fn = loss_fn
        self.regul_rate = regul_rate
        self.rel_total = self.model.num_relations if model is not None else 237
        self.neg_ent = neg_ent
        self.bern_flag = bern_flag
        self.filter_flag = filter_flag
        self.sampling_mode = sampling_mode
        self.score_norm_flag = score_norm_flag
        self.p_norm = 1
        self.dim = self.model.dim if model is not None else None
        self.whole_triples = whole_triples
        self.seed = seed
        self._sampler = None

    def get_model_device(self):
        return next(self.parameters()).device if any(True for _ in self.parameters()) else torch.device("cuda:0")

    def sampler(self, device):
        if self._sampler is None:
            h, r, t = self.whole_triples
            self._sampler = RepoSampler([h, r, t], self.rel_total, device, filter_flag=self.filter_flag,
                                        seed=self.seed)
        return self._sampler

    def neg_sample_fn(self, local_global_id, node_list, edge_index, edge_type):
        """-> (2, B(1+k)) and (B(1+k),) int tensors in the layout [pos | neg_1 | ... | neg_k]."""
        dev = edge_index.device if edge_index.is_cuda else torch.device("cuda:0")
        n_local = int(len(node_list))
        l2g = None
        if local_global_id is not None:
            l2g = torch.as_tensor([local_global_id[i] for i in range(n_local)], dtype=torch.int64)
        ei, et = self.sampler(dev).sample(edge_index.to(dev), edge_type.to(dev), self.neg_ent, n_local, l2g)
        return ei, et

    def _spec(self, score_model, dim):
        if score_model == "transe":
            return NSSpec("transe", dim, norm_flag=self.score_norm_flag)
        if score_model == "distmult":
            return NSSpec("distmult", dim)
        raise ValueError("invalid scoring model!")

    def _calc(self, h, t, r, mode="normal", score_model="transe"):
        """Score rows of explicit vectors (NegativeSampling.py:142-168): rows are gathered as
        tables indexed by arange."""
        n = h.shape[0]
        dev = h.device
        idx = torch.arange(n, device=dev)
        tab = torch.cat([h, t], 0).contiguous()
        return score_rows(self._spec(score_model, h.shape[-1]), tab, r.contiguous(), idx, idx + n, idx)

    def scoring_fn(self, local_global_id, x, relations, edge_index, edge_type):
        n = relations.shape[0]
        idx = torch.arange(n, device=x.device)
        return score_rows(self._spec("transe", x.shape[-1]), x, relations, edge_index[0].long(),
                          edge_index[1].long(), idx)

    def _get_positive_score(self, score, num_pos_samples):
        return score[:num_pos_samples].view(-1, num_pos_samples).permute(1, 0)

    def _get_negative_score(self, score, num_pos_samples):
        return score[num_pos_samples:].view(-1, num_pos_samples).permute(1, 0)

    def struct_loss(self, x_gcn, rel_emb, edge_index_expand, num_pos):
        """Fused margin loss + regul_rate * regularization over the expanded edges."""
        dev = x_gcn.device
        B = int(num_pos)
        k = int(edge_index_expand.shape[1]) // B - 1
        r = torch.arange(B, device=dev).repeat(1 + k)
        margin, adv = self.loss_fn.fused_args()
        loss, score = fused_ns_loss(self._spec("transe", x_gcn.shape[-1]), x_gcn.contiguous(), rel_emb.contiguous(),
                                    edge_index_expand[0].to(dev).long(), edge_index_expand[1].to(dev).long(), r, B,
                                    k, margin, adv, self.regul_rate)
        return loss, score

    def forward(self, local_global_id, edge_index, edge_type, batch, deterministic=False):
        x_gcn, rel_emb, batch_output = self.model(edge_index, edge_type, batch, deterministic)
        mapped_node_list = torch.arange(int(torch.max(edge_index)))
        ei, et = self.neg_sample_fn(local_global_id, mapped_node_list, edge_index, edge_type)
        loss_res_gcn, _ = self.struct_loss(x_gcn, rel_emb, ei, len(edge_type))
        struct_loss = loss_res_gcn  # aliasing of the reference: regul already folded in (P9)
        a = self.args
        image_loss = batch_output.get("image_loss", 0.0)
        text_loss = batch_output.get("text_loss", 0.0)
        contrastive_loss = batch_output.get("contrastive_loss", 0.0)
        loss_image_text = a.image_loss_weight * image_loss + a.text_loss_weight * text_loss
        loss = loss_image_text + a.gcn_loss_weight * loss_res_gcn + a.contrastive_loss_weight * contrastive_loss
        info = dict(struct_loss=struct_loss, gcn_loss=loss_res_gcn, loss_image_text=loss_image_text,
                    image_loss=image_loss, text_loss=text_loss, contrastive_loss=contrastive_loss)
        return loss, info

    def evaluate(self, h, r, t, score_model="transe"):
        """(h + r) - t, L1, optional normalisation (NegativeSampling.py:294-305)."""
        if score_model != "transe":
            print("invalid scoring model!")
            return None
        return self._calc(h, t, r, score_model="transe")

    def regularization(self, x, relations, edge_index, edge_type):
        bh = x[edge_index[0].long()]
        bt = x[edge_index[1].long()]
        return (torch.mean(bh ** 2) + torch.mean(bt ** 2) + torch.mean(relations ** 2)) / 3

    def generate_eval_list(self, local_global_id, edge_index, edge_type):
        mapped_node_list = torch.arange(int(torch.max(edge_index)))
        return self.neg_sample_fn(local_global_id, mapped_node_list, edge_index, edge_type)
