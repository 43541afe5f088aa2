"""zsl_extractor.py -- TEST INFRASTRUCTURE ONLY: oracle for the ZSL Extractor path.

Only ``tests/`` import this module, as the checker; the product package never does.
A plain torch-fp32 (CPU) restatement, operation for operation, of

* ``Extractor.neighbor_encoder`` / ``entity_encoder`` / ``forward``
  (``module/zsl_module.py:47-110``) with ``SupportEncoder`` (``module/submodule.py:240-258``),
  eval mode (dropout = identity);
* ``ZSLmodule.load_embed`` (``zsl_module.py:208-232``), ``build_connection`` (:233-263),
  ``get_meta`` (:265-287) as literal per-element Python loops;
* the ranking of ``ZSLmodule.eval`` (:666-706): sklearn ``cosine_similarity`` of the
  candidate vectors with the generated relation vectors, ``mean(axis=1)``, rank of row 0 in
  ``argsort(scores)[::-1]``.

Parity status: **unpinned by reference fixtures**. No golden vectors of the Extractor exist in
the reference, and running the reference's own Python to produce them is denied in this
pipeline, so this restatement -- written from the reference's source text -- is
the oracle. The product path (csrc/extractor.hip) reassociates the computation (per-node
tables, sum-then-project neighbour encoder, MFMA accumulation), so parity is by tolerance
(1e-4) on vectors and scores, and exact on ranks for tie-free candidate lists.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class SupportEncoderRef(nn.Module):
    def __init__(self, d_model, d_inner):
        super().__init__()
        self.proj1 = nn.Linear(d_model, d_inner)
        self.proj2 = nn.Linear(d_inner, d_model)
        self.layer_norm = nn.LayerNorm(d_model)

    def forward(self, x):  # submodule.py:254-258 (dropout = identity in eval)
        return self.layer_norm(self.proj2(F.relu(self.proj1(x))) + x)


class ExtractorRef(nn.Module):
    """Same parameter names as the reference Extractor, so state_dicts move both ways."""

    def __init__(self, embed_dim, num_symbols, embed):
        super().__init__()
        d = int(embed_dim)
        self.embed_dim = d
        self.symbol_emb = nn.Embedding(num_symbols + 1, d, padding_idx=num_symbols)
        self.symbol_emb.weight.data.copy_(torch.as_tensor(np.asarray(embed), dtype=torch.float32))
        self.gcn_w = nn.Linear(d, d // 2)
        self.gcn_b = nn.Parameter(torch.zeros(d))
        self.fc1 = nn.Linear(d, d // 2)
        self.fc2 = nn.Linear(d, d // 2)
        self.reshape_layer = nn.Linear(2 * d, d)
        self.support_encoder = SupportEncoderRef(d, 2 * d)

    def neighbors(self, connections, num_neighbors):  # :47-59
        ent = self.symbol_emb(connections[:, :, 1])            # (B, max, d)
        out = self.gcn_w(ent).sum(dim=1)                       # per-slot Linear, then the slot sum
        return (out / num_neighbors.unsqueeze(1)).tanh()

    def entities(self, e1, e2):  # :61-67
        return torch.cat((self.fc1(e1), self.fc2(e2)), dim=-1).tanh()

    def encode(self, pairs, meta):  # :80-99 for one side
        lc, ld, rc, rd = meta
        ent = self.entities(self.symbol_emb(pairs[:, 0]), self.symbol_emb(pairs[:, 1]))
        x = torch.cat((self.neighbors(lc, ld), ent, self.neighbors(rc, rd)), dim=-1)
        return self.support_encoder(self.reshape_layer(x))

    @torch.no_grad()
    def forward(self, query, support, query_meta, support_meta):  # :69-104
        q = self.encode(query, query_meta)
        s = self.encode(support, support_meta).mean(dim=0, keepdim=True)
        return q, torch.matmul(q, s.t()).squeeze()


def load_embed(rel2id, ent2id, ent_embed, rel_embed):
    """zsl_module.py:208-232, element by element."""
    symbol_id, i, embeddings = {}, 0, []
    for key in rel2id.keys():
        if key not in ["", "OOV"]:
            symbol_id[key] = i
            i += 1
            embeddings.append(list(rel_embed[rel2id[key], :]))
    for key in ent2id.keys():
        if key not in ["", "OOV"]:
            symbol_id[key] = i
            i += 1
            embeddings.append(list(ent_embed[ent2id[key], :]))
    symbol_id["PAD"] = i
    embeddings.append(list(np.zeros((rel_embed.shape[1],))))
    return symbol_id, np.array(embeddings)


def build_connection(train_tasks, test_tasks, ent2id, symbol2id, pad_id, max_):
    """zsl_module.py:233-263, element by element."""
    conns = (np.ones((len(ent2id), max_, 2)) * pad_id).astype(int)
    e1_rele2 = defaultdict(list)
    e1_degrees = defaultdict(int)
    for tasks in (train_tasks, test_tasks):
        for rel in tasks.keys():
            for tri in tasks[rel]:
                e1, r, e2 = tri
                e1_rele2[e1].append((symbol2id[r], symbol2id[e2]))
                e1_rele2[e2].append((symbol2id[r], symbol2id[e1]))
    for ent, id_ in ent2id.items():
        neighbors = e1_rele2[ent]
        if len(neighbors) > max_:
            neighbors = neighbors[:max_]
        e1_degrees[id_] = len(neighbors)
        for idx, nb in enumerate(neighbors):
            conns[id_, idx, 0] = nb[0]
            conns[id_, idx, 1] = nb[1]
    return conns, e1_degrees


def get_meta(connections, e1_degrees, left, right):
    """zsl_module.py:265-287."""
    return (torch.LongTensor(np.stack([connections[_, :, :] for _ in left], axis=0)),
            torch.FloatTensor([e1_degrees[_] for _ in left]),
            torch.LongTensor(np.stack([connections[_, :, :] for _ in right], axis=0)),
            torch.FloatTensor([e1_degrees[_] for _ in right]))


def zsl_eval_ranks(extractor, symbol2id, ent2id, connections, e1_degrees, relation_vecs, test_candidates):
    """ZSLmodule.eval's per-query loop (zsl_module.py:655-706) for a dict of generated relation
    vectors {rel: (S, d) numpy}. Returns (ranks, scores per query)."""
    from sklearn.metrics.pairwise import cosine_similarity
    ranks, all_scores = [], []
    for query_ in test_candidates.keys():
        rv = np.asarray(relation_vecs[query_], np.float32)
        for e1_rel, tail_candidates in test_candidates[query_].items():
            head = e1_rel.split("\t")[0]
            pairs = [[symbol2id[head], symbol2id[c]] for c in tail_candidates]
            left = [ent2id[head]] * len(tail_candidates)
            right = [ent2id[c] for c in tail_candidates]
            q = torch.LongTensor(pairs)
            meta = get_meta(connections, e1_degrees, left, right)
            vecs, _ = extractor(q, q, meta, meta)
            scores = cosine_similarity(vecs.numpy(), rv).mean(axis=1)
            order = list(np.argsort(scores))[::-1]
            ranks.append(order.index(0) + 1)
            all_scores.append(scores)
    return np.asarray(ranks), all_scores


# ------------------------------------------------------------------ pretraining (training mode) --
def train_encode_ref(ref, pairs, meta, masks, p=0.2):
    """Training-mode Extractor rows (zsl_module.py:47-99 with SupportEncoder submodule.py:254-258),
    every nn.Dropout replaced by its given 0/1 mask: dropout(x) = x * mask / (1 - p). Literal op
    order of the reference: per-slot gcn_w then the slot sum. masks = (nb_left (B, M, d),
    nb_right (B, M, d), ent (B, 2, d), support_encoder (B, d))."""
    nb_l, nb_r, ent_m, se_m = (torch.as_tensor(np.asarray(m)).to(ref.gcn_w.weight.dtype) for m in masks)
    scale = 1.0 / (1.0 - p)
    lc, ld, rc, rd = meta
    w = ref.gcn_w.weight.dtype

    def nb(conn, deg, m):                                       # :47-59
        e = ref.symbol_emb(conn[:, :, 1]) * (m * scale)
        return (ref.gcn_w(e).sum(dim=1) / deg.to(w).unsqueeze(1)).tanh()

    e1 = ref.symbol_emb(pairs[:, 0]) * (ent_m[:, 0] * scale)  # :61-67
    e2 = ref.symbol_emb(pairs[:, 1]) * (ent_m[:, 1] * scale)
    ent = torch.cat((ref.fc1(e1), ref.fc2(e2)), dim=-1).tanh()
    x = ref.reshape_layer(torch.cat((nb(lc, ld, nb_l), ent, nb(rc, rd, nb_r)), dim=-1))
    se = ref.support_encoder
    y = se.proj2(F.relu(se.proj1(x))) * (se_m * scale)
    return se.layer_norm(y + x)


def pretrain_step_ref(ref, pairs, meta, sizes, masks, margin, lr, p=0.2):
    """One pretrain_Extractor step (zsl_module.py:296-344) on rows [support | query | support |
    false] (sizes = (S, Q, F)): the two Extractor calls' query / false scores against their own
    support means (:318-323), loss relu(margin - (q - f)).mean() (:325-326), backward and one
    torch.optim.Adam step (lr, default betas; optim_E :183-186). Returns (loss, grads {name:
    tensor}, updated parameters {name: tensor}); run it on a float64 copy for a float64 oracle."""
    S, Q, F_ = sizes
    params = {n: q for n, q in ref.named_parameters() if q.requires_grad and not n.startswith("symbol_emb")}
    opt = torch.optim.Adam(list(params.values()), lr=lr)
    opt.zero_grad()
    g = train_encode_ref(ref, pairs, meta, masks, p)
    s1 = g[:S].mean(dim=0, keepdim=True)
    s2 = g[S + Q:2 * S + Q].mean(dim=0, keepdim=True)
    qs = torch.matmul(g[S:S + Q], s1.t()).squeeze()
    fs = torch.matmul(g[2 * S + Q:], s2.t()).squeeze()
    loss = F.relu(margin - (qs - fs)).mean()
    loss.backward()
    grads = {n: (None if q.grad is None else q.grad.detach().clone()) for n, q in params.items()}
    opt.step()
    return loss.detach(), grads, {n: q.detach().clone() for n, q in params.items()}
