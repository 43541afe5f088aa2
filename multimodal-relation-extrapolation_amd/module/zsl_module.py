"""Zero-shot evaluation path of ZSLmodule (module/zsl_module.py): the Extractor
(:17-110), the symbol / neighbourhood tables it reads (load_embed :208-232,
build_connection :233-263, get_meta :265-287) and the evaluation ranking of
ZSLmodule.eval (:635-745).

* `Extractor(embed_dim, num_symbols, embed)` keeps the reference's constructor, parameter
  names (state_dict-compatible) and `forward(query, support, query_meta, support_meta) ->
  (query_g, matching_scores)`. In eval mode forward runs on the GPU (csrc/extractor.hip):
  per-row neighbour / entity encoders folded through reshape_layer, then the SupportEncoder
  on MFMA. In training mode (the three nn.Dropout(0.2)) it runs the pretraining step's
  launch chain (mmre.extractor_train: dropped neighbour sums gathered on the GPU, the linears
  on the split-K GEMM, counter-hash dropout masks).
* `ZSLGraph` builds symbol2id / symbol2vec / connections / e1_degrees exactly as the
  reference does, with numpy instead of per-element Python loops.
* `ZSLEvaluator.eval(relation_vecs, test_candidates)` is ZSLmodule.eval's ranking for every
  query at once: Extractor vectors of all candidate pairs, mean cosine similarity with the
  relation's generated vectors, rank of the true tail, Hits@10/5/1 and MRR printed as the
  reference prints them.
* `zsl_rank` ranks precomputed candidate vectors (csrc/candidates.hip).
* `ZSLmodule(args, data_path, r2id, e2id, device, dataset)` is the reference's class
  (:140-790) over the pieces above: `update_embed`, `get_meta`, `train(generate_model)` (the
  adversarial loop on mmre.gan.ZSLGANStep, hipGraph-replayed D / G steps, then save + eval),
  `eval(generate_model, mode, meta, load_pretrain)` -> (hits10, hits5, mrr) with every
  relation's generate() in one batched call and every candidate ranked in one launch
  sequence, `save` / `load` / `save_pretrain` / `load_pretrain`, and the Extractor's own
  pretraining (`pretrain_Extractor`, :289-348: margin loss over dropped-out Extractor vectors,
  torch Adam) through mmre.extractor_train.PretrainStep, captured once per batch shape into a
  hipGraph.
"""
import json
import os
from collections import defaultdict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from mmre._lib import MMREError
from mmre.candidates import cosine_rank
from mmre.extractor import ZSLRanker, _check_ids, encode, node_tables, pack_weights, targets
from mmre.gemm import layer_norm, mm, sn_linear
from .submodule import LayerNormalization, SupportEncoder
from .utils import weights_init  # noqa: F401  (module/utils.py:119-123; re-exported, zsl_module imports utils *)


class Extractor(nn.Module):
    """Matching metric based on KB embeddings (zsl_module.py:17-110)."""

    def __init__(self, embed_dim, num_symbols, embed=None):
        super().__init__()
        self.embed_dim = int(embed_dim)
        self.pad_idx = num_symbols
        self.symbol_emb = nn.Embedding(num_symbols + 1, embed_dim, padding_idx=num_symbols)
        self.num_symbols = num_symbols
        self.gcn_w = nn.Linear(self.embed_dim, int(self.embed_dim / 2))
        self.gcn_b = nn.Parameter(torch.zeros(self.embed_dim))  # declared, unused by forward (as in :29)
        self.fc1 = nn.Linear(self.embed_dim, int(self.embed_dim / 2))
        self.fc2 = nn.Linear(self.embed_dim, int(self.embed_dim / 2))
        self.dropout = nn.Dropout(0.2)
        self.dropout_e = nn.Dropout(0.2)
        if embed is not None:
            self.symbol_emb.weight.data.copy_(torch.as_tensor(np.asarray(embed), dtype=torch.float32))
        self.symbol_emb.weight.requires_grad = False
        self.reshape_layer = nn.Linear(self.embed_dim * 2, self.embed_dim)
        self.support_encoder = SupportEncoder(self.embed_dim, 2 * self.embed_dim, dropout=0.2)

    def _require_eval(self):
        if self.training:
            raise MMREError("Extractor.encode_pairs is the eval-mode encoder (training mode goes through "
                            "forward(), mmre.extractor_train): call .eval()")

    def encode_pairs(self, pairs, meta, targets_=None, normalize=False, want_g=True):
        """query_g (and optionally scores vs targets_) of (B, 2) symbol pairs with their meta."""
        self._require_eval()
        left_conn, left_deg, right_conn, right_deg = meta
        n_sym = int(self.symbol_emb.weight.shape[0])
        for ids, what in ((pairs, "symbol ids"), (left_conn[:, :, 1], "left neighbours"),
                          (right_conn[:, :, 1], "right neighbours")):
            _check_ids(ids, n_sym, what)
        d = self.embed_dim
        pack = pack_weights(self)
        emb = self.symbol_emb.weight
        left, _ = node_tables(pack, d, emb, pairs[:, 0], left_conn, left_deg, want_right=False)
        _, right = node_tables(pack, d, emb, pairs[:, 1], right_conn, right_deg, want_left=False)
        idx = torch.arange(pairs.shape[0], device=pairs.device)
        return encode(pack, d, self.support_encoder.layer_norm.eps, left, idx, right, idx, targets=targets_,
                      normalize=normalize, want_g=want_g, want_score=targets_ is not None)

    def forward(self, query, support, query_meta=None, support_meta=None):
        """query (B, 2), support (few, 2) symbol ids; metas from ZSLGraph.get_meta.
        Returns (query_g (B, d), matching_scores = query_g . mean(support_g) squeezed).
        Training mode: differentiable, dropout masks drawn per call (one launch chain over the
        support and query rows together)."""
        if self.training:
            from mmre.extractor_train import DropoutRNG, train_forward
            if getattr(self, "_rng", None) is None or self._rng.state.device != query.device:
                self._rng = DropoutRNG(torch.initial_seed(), query.device)
            S = int(support.shape[0])
            pairs = torch.cat((support, query))
            meta = tuple(torch.cat((a, b)) for a, b in zip(support_meta, query_meta))
            g = train_forward(self, pairs, meta, rng=self._rng)
            self._rng.advance()
            query_g = g[S:]
            return query_g, torch.matmul(query_g, g[:S].mean(0, keepdim=True).t()).squeeze()
        support_g, _ = self.encode_pairs(support, support_meta)
        s_mean = targets(support_g.unsqueeze(0), normalize=False)  # (1, d) = mean over support rows
        query_g, scores = self.encode_pairs(query, query_meta, targets_=s_mean, normalize=False)
        return query_g, scores.unsqueeze(1).squeeze()

    def update(self, embed):
        self.symbol_emb.weight.data.copy_(torch.as_tensor(np.asarray(embed), dtype=torch.float32))
        self.symbol_emb.weight.requires_grad = False


class Discriminator(nn.Module):
    """Discriminator (zsl_module.py:112-138): spectral-normalised fc_middle (d -> d, leaky_relu,
    LayerNormalization) shared by the sample and the class centroids, spectral-normalised fc_TF
    (d -> 1) for the WGAN critic, and class scores against the centroids. Same parameter and
    buffer names (fc_middle.weight_orig / weight_u / weight_v / bias, fc_TF.*, layer_norm.a_2 /
    b_2). Runs as autograd on the device inside the GAN step's hipGraph (mmre.gan) with its
    pieces on HIP kernels (mmre.gemm): the spectral-norm weight (power iteration, sigma, W /
    sigma) in one launch per call, the products x W^T + b and the class scores -- and all their
    derivatives, the gradient penalty's double backward included -- on the split-K GEMM, the
    LayerNormalization forward and first-order backward in HIP; leaky_relu stays a torch op."""

    def __init__(self, dropout=0.3, dim=200):
        super().__init__()
        self.fc_middle = nn.utils.spectral_norm(nn.Linear(dim, dim))
        self.fc_TF = nn.utils.spectral_norm(nn.Linear(dim, 1))
        self.layer_norm = LayerNormalization(dim)

    def forward(self, ep_vec, centroid_matrix):
        middle_vec = layer_norm(self.layer_norm, F.leaky_relu(sn_linear(self.fc_middle, ep_vec)))
        centroid_matrix = layer_norm(self.layer_norm, F.leaky_relu(sn_linear(self.fc_middle, centroid_matrix)))
        logit_TF = sn_linear(self.fc_TF, middle_vec)
        class_scores = mm(middle_vec, centroid_matrix.t())
        return middle_vec, logit_TF, class_scores


class ZSLGraph:
    """Symbol tables and neighbourhoods of ZSLmodule (zsl_module.py:208-287).

    rel2id / ent2id: the id maps (dict name -> id, iteration order matters: symbols are
    numbered relations first, then entities, skipping "" and "OOV", PAD last); train_tasks /
    test_tasks: {relation: [[e1, rel, e2], ...]}; ent_embs (n_nodes, d), rel_embs (n_rel, d)."""

    def __init__(self, rel2id, ent2id, train_tasks, test_tasks, ent_embs, rel_embs, max_neighbor=50):
        self.rel2id, self.ent2id = rel2id, ent2id
        self.load_embed(ent_embs, rel_embs)
        self.num_symbols = len(self.symbol2id) - 1
        self.pad_id = self.num_symbols
        self.num_ents = len(ent2id)
        self.build_connection(train_tasks, test_tasks, max_=max_neighbor)

    def load_embed(self, ent_embs, rel_embs):
        """load_embed (:208-232)."""
        ent = np.asarray(ent_embs.detach().cpu() if torch.is_tensor(ent_embs) else ent_embs)
        rel = np.asarray(rel_embs.detach().cpu() if torch.is_tensor(rel_embs) else rel_embs)
        rel_keys = [k for k in self.rel2id if k not in ("", "OOV")]
        ent_keys = [k for k in self.ent2id if k not in ("", "OOV")]
        self.symbol2id = {k: i for i, k in enumerate(rel_keys + ent_keys)}
        self.symbol2id["PAD"] = len(rel_keys) + len(ent_keys)
        rows = [rel[[self.rel2id[k] for k in rel_keys]].reshape(len(rel_keys), rel.shape[1]),
                ent[[self.ent2id[k] for k in ent_keys]].reshape(len(ent_keys), rel.shape[1]),
                np.zeros((1, rel.shape[1]))]
        # the reference builds a float64 array from python lists of float32 values
        self.symbol2vec = np.concatenate(rows, 0).astype(np.float64)

    def build_connection(self, train_tasks, test_tasks, max_=100):
        """build_connection (:233-263): each triple adds (rel, e2) to e1's list and (rel, e1)
        to e2's, train tasks first then test tasks, in file order; lists cut at max_."""
        s2i = self.symbol2id
        nbrs = defaultdict(list)
        for tasks in (train_tasks, test_tasks):
            for rel in tasks.keys():
                for e1, r, e2 in tasks[rel]:
                    nbrs[e1].append((s2i[r], s2i[e2]))
                    nbrs[e2].append((s2i[r], s2i[e1]))
        conn = np.full((self.num_ents, max_, 2), self.pad_id, dtype=np.int64)
        deg = np.zeros(self.num_ents, dtype=np.int64)
        for ent, id_ in self.ent2id.items():
            lst = nbrs.get(ent, [])[:max_]
            deg[id_] = len(lst)
            if lst:
                conn[id_, :len(lst)] = np.asarray(lst, dtype=np.int64)
        self.connections = conn
        self.e1_degrees = deg
        # symbol id of every entity id (ids of "" / "OOV" map to PAD)
        self.ent_sym = np.full(self.num_ents, self.pad_id, dtype=np.int64)
        for ent, id_ in self.ent2id.items():
            if ent in s2i:
                self.ent_sym[id_] = s2i[ent]
        return {ent: int(deg[id_]) for ent, id_ in self.ent2id.items()}

    def get_meta(self, left, right, device=None):
        """get_meta (:265-287): (left_connections, left_degrees, right_connections, right_degrees)."""
        left, right = np.asarray(left, np.int64), np.asarray(right, np.int64)
        to = lambda a, dt: torch.as_tensor(a, dtype=dt, device=device)
        return (to(self.connections[left], torch.int64), to(self.e1_degrees[left], torch.float32),
                to(self.connections[right], torch.int64), to(self.e1_degrees[right], torch.float32))


class ZSLEvaluator:
    """ZSLmodule.eval's ranking (zsl_module.py:666-745) for all queries at once."""

    def __init__(self, extractor: Extractor, graph: ZSLGraph, device=None):
        extractor.eval()
        self.graph = graph
        self.ranker = ZSLRanker(extractor, graph.ent_sym, graph.connections, graph.e1_degrees, device=device)

    def flatten(self, test_candidates, rel_order=None):
        """test_candidates {rel: {"head\\trel\\ttrue": [true, cand...]}} -> device CSR of
        (head id, tail id) rows, query -> relation-set index, and the relation order."""
        e2id = self.graph.ent2id
        rels = list(test_candidates.keys()) if rel_order is None else list(rel_order)
        heads, tails, off, qset, qrel = [], [], [0], [], []
        for ri, rel in enumerate(rels):
            for e1_rel, cands in test_candidates[rel].items():
                head = e1_rel.split("\t")[0]
                h = e2id[head]
                ids = [e2id[c] for c in cands]
                heads.append(np.full(len(ids), h, np.int64))
                tails.append(np.asarray(ids, np.int64))
                off.append(off[-1] + len(ids))
                qset.append(ri)
                qrel.append(rel)
        dev = self.ranker.left.device
        to = lambda a: torch.as_tensor(np.concatenate(a) if isinstance(a, list) else a, device=dev)
        return (to(heads), to(tails), torch.as_tensor(np.asarray(off, np.int64), device=dev),
                torch.as_tensor(np.asarray(qset, np.int64), device=dev), rels, qrel)

    def rank(self, relation_vecs, test_candidates, rel_order=None, return_scores=False):
        """relation_vecs: {rel: (test_sample, d)} generated vectors (generate_model.generate,
        :660-666) or a (n_rel, S, d) tensor in rel_order. Returns int32 ranks per query in
        test_candidates order (and the query relations)."""
        ch, ct, off, qset, rels, qrel = self.flatten(test_candidates, rel_order)
        if isinstance(relation_vecs, dict):
            rv = torch.stack([torch.as_tensor(relation_vecs[r]) for r in rels]).float()
        else:
            rv = torch.as_tensor(relation_vecs).float()
        out = self.ranker.rank(ch, ct, off, rv, qset, return_scores=return_scores)
        return out, qrel

    def eval(self, relation_vecs, test_candidates, mode="test"):
        (ranks, _), qrel = self.rank(relation_vecs, test_candidates, return_scores=True)
        r = ranks.cpu().numpy()
        per_rel = {}
        qrel = np.asarray(qrel, dtype=object)
        for rel in dict.fromkeys(qrel):
            per_rel[rel] = qrel == rel
        return zsl_metrics(r, mode, per_relation=per_rel)


def train_generate_decription(train_tasks, rel2candidates, e1rel_e2, ent2id, rel2id, rela2label, batch_size,
                              gan_batch_rela, rng=None):
    """Batch generator of ZSLmodule.train (module/utils.py:625-689) as id arrays: per batch,
    gan_batch_rela shuffled train relations with > 20 candidates, batch_size query triples each
    (with replacement when the relation has fewer), one false tail per query drawn from the
    relation's candidates (known to ent2id, not a known tail of (head, rel), not the true tail).
    Yields dict(rel, q_head, q_tail, f_head, f_tail, labels) of int64 numpy arrays: relation id
    per row (the description row, utils.py:686), entity ids (ent2id) and label ids. Draws come
    from `rng` (a random.Random; the reference uses the unseeded module-level `random`)."""
    import random as _random
    rng = rng if rng is not None else _random.Random()
    pool = list(train_tasks.keys())
    while True:
        out = {k: [] for k in ("rel", "q_head", "q_tail", "f_head", "f_tail", "labels")}
        rng.shuffle(pool)
        for query in pool[:gan_batch_rela]:
            cands = rel2candidates[query]
            if len(cands) <= 20:
                continue
            triples = list(train_tasks[query])
            rng.shuffle(triples)
            if not triples:
                continue
            picked = ([rng.choice(triples) for _ in range(batch_size)] if len(triples) < batch_size
                      else rng.sample(triples, batch_size))
            for h, r, t in picked:
                while True:
                    noise = rng.choice(cands)
                    if noise in ent2id and noise not in e1rel_e2[h + r] and noise != t:
                        break
                out["rel"].append(rel2id[query])
                out["q_head"].append(ent2id[h])
                out["q_tail"].append(ent2id[t])
                out["f_head"].append(ent2id[h])
                out["f_tail"].append(ent2id[noise])
                out["labels"].append(rela2label[query])
        yield {k: np.asarray(v, np.int64) for k, v in out.items()}


def gan_train(step, batches, train_times, D_epoch=1, G_epoch=1, loss_every=50, device=None, graphs=True):
    """The loop of ZSLmodule.train (zsl_module.py:417-609) over `batches` (an iterator of
    train_generate_decription dicts) with a mmre.gan.ZSLGANStep; prints the reference's
    'Epoch: ...' line every loss_every epochs. Each D / G step replays its hipGraph."""
    from collections import deque
    D_every, G_every = D_epoch * loss_every, G_epoch * loss_every
    D_losses = deque([], D_every)
    G_losses = deque([], G_every)
    dev = device if device is not None else step.device
    for epoch in range(train_times):
        for _ in range(D_epoch):
            b = {k: torch.as_tensor(v, device=dev) for k, v in next(batches).items()}
            d = step.replay("d", b) if graphs else step.d_step(
                b["rel"], b["q_head"], b["q_tail"], b["f_head"], b["f_tail"], b["labels"],
                torch.randn(len(b["rel"]), step.G.noise_dim, device=dev), torch.rand(len(b["rel"]), 1, device=dev))
            D_losses.append(d.detach().cpu().numpy().copy())
        for _ in range(G_epoch):
            b = {k: torch.as_tensor(v, device=dev) for k, v in next(batches).items()}
            g = step.replay("g", b) if graphs else step.g_step(
                b["rel"], b["q_head"], b["q_tail"], b["f_head"], b["f_tail"], b["labels"],
                torch.randn(len(b["rel"]), step.G.noise_dim, device=dev))
            G_losses.append(g.detach().cpu().numpy().copy())
        if epoch % loss_every == 0 and epoch != 0:
            Dm, Gm = np.mean(D_losses, 0), np.mean(G_losses, 0)
            # D: loss, real, real-class, fake, fake-class; G: loss, fake, class, real-class, VP
            print("Epoch: %d, D_loss: %.2f [%.2f, %.2f, %.2f, %.2f], G_loss: %.2f [%.2f, %.2f, %.2f, %.2f]"
                  % (epoch, Dm[0], Dm[1], Dm[2], Dm[3], Dm[4], Gm[0], Gm[1], Gm[2], Gm[3], Gm[4]))
    return step


def zsl_rank(candidate_vecs, cand_off, relation_vecs, rel_of_query):
    return cosine_rank(candidate_vecs, cand_off, relation_vecs, rel_of_query)


def zsl_metrics(ranks, mode="test", per_relation=None):
    r = np.asarray(ranks)
    h10 = (r <= 10).astype(float)
    h5 = (r <= 5).astype(float)
    h1 = (r <= 1).astype(float)
    mrr = 1.0 / r
    if per_relation is not None:
        for name, sel in per_relation.items():
            print("{} Hits10:{:.3f}, Hits5:{:.3f}, Hits1:{:.3f} MRR:{:.3f}".format(
                mode + name, h10[sel].mean(), h5[sel].mean(), h1[sel].mean(), mrr[sel].mean()))
    print("############   " + mode + "    #############")
    print("HITS10: {:.3f}".format(h10.mean()))
    print("HITS5: {:.3f}".format(h5.mean()))
    print("HITS1: {:.3f}".format(h1.mean()))
    print("MAP: {:.3f}".format(mrr.mean()))
    print("###################################")
    return float(h10.mean()), float(h5.mean()), float(mrr.mean())


def _read_json(path):
    with open(path) as f:
        return json.load(f)


class ZSLmodule(nn.Module):
    """ZSLmodule (zsl_module.py:140-790). data_path holds the reference's files:
    train_tasks_zsl.json, test_tasks_zsl.json, rel2candidates_all.json, e1rel_e2_all.json and
    <mode>_candidates.json for eval; dataset provides generate_batch([], relation ids) ->
    rel_des / rel_des_padding_mask (module.data.ZSDataset), num_nodes and num_relations."""

    def __init__(self, args, data_path, r2id, e2id, device, dataset, pretrain_margin=3.0):
        super().__init__()
        for k, v in vars(args).items():
            if not hasattr(nn.Module, k):  # the reference's setattr would shadow nn.Module.cuda etc.
                setattr(self, k, v)
        self.args = args
        self.data_path = data_path
        self.train_tasks = _read_json(os.path.join(data_path, "train_tasks_zsl.json"))
        self.test_tasks = _read_json(os.path.join(data_path, "test_tasks_zsl.json"))
        self.rel2id = r2id
        self.ent2id = e2id
        self.device = torch.device(device)
        self.prertain_margin = pretrain_margin  # (sic, :151) stored, unused by the reference as well
        self.rel2candidates = _read_json(os.path.join(data_path, "rel2candidates_all.json"))
        self.e1rel_e2 = _read_json(os.path.join(data_path, "e1rel_e2_all.json"))
        self.test_noises = 0.1 * torch.randn(self.test_sample, self.noise_dim).to(self.device)
        self.meta = not self.no_meta
        self.label_num = len(self.train_tasks.keys())
        batch_data = dataset.generate_batch([], torch.arange(0, len(self.rel2id)))
        self.des_tokens, self.des_pad_masks = batch_data["rel_des"], batch_data["rel_des_padding_mask"]
        self.rela2label = {rela: i for i, rela in enumerate(sorted(self.train_tasks.keys()))}
        ent_embs = torch.rand((dataset.num_nodes, self.emb_dim))
        rel_embs = torch.rand((dataset.num_relations, self.emb_dim))
        print("##LOADING PRE-TRAINED EMBEDDING")
        print("##BUILDING CONNECTION MATRIX")
        self.graph = ZSLGraph(r2id, e2id, self.train_tasks, self.test_tasks, ent_embs, rel_embs,
                              max_neighbor=self.max_neighbor)
        self.num_symbols = self.graph.num_symbols
        self.pad_id = self.num_symbols
        self.num_ents = len(self.ent2id.keys())
        self.Extractor = Extractor(self.emb_dim, self.num_symbols, embed=self.graph.symbol2vec)
        self.Extractor.to(self.device)
        self.Extractor.apply(weights_init)
        self.Discriminator = Discriminator(dim=self.emb_dim)
        self.Discriminator.to(self.device)
        self.Discriminator.apply(weights_init)
        self.centroid_matrix = None
        self.gan_step = None

    # symbol tables (load_embed / build_connection, :209-268)
    @property
    def symbol2id(self):
        return self.graph.symbol2id

    @property
    def symbol2vec(self):
        return self.graph.symbol2vec

    @property
    def connections(self):
        return self.graph.connections

    @property
    def e1_degrees(self):
        return self.graph.e1_degrees

    def load_embed(self, ent_embs, rel_embs):
        print("##LOADING PRE-TRAINED EMBEDDING")
        self.graph.load_embed(ent_embs, rel_embs)

    def update_embed(self, ent_embs, rel_embs):
        """:235-237: new symbol table from the entity / relation embeddings, into the Extractor."""
        self.load_embed(ent_embs, rel_embs)
        self.Extractor.update(self.graph.symbol2vec)

    def get_meta(self, left, right):
        return self.graph.get_meta(left, right, device=self.device)

    # ---------------------------------------------------------------- training
    def _pretrain_step(self):
        """optim_E (Adam, lr_E) persists across train() calls, as the reference's (:183-186)."""
        if getattr(self, "_pstep", None) is None:
            from mmre.extractor_train import PretrainStep
            dev = self.device
            g = self.graph
            self._pstep = PretrainStep(self.Extractor, torch.as_tensor(g.ent_sym, device=dev),
                                       torch.as_tensor(g.connections, device=dev),
                                       torch.as_tensor(g.e1_degrees, dtype=torch.float32, device=dev),
                                       lr=self.lr_E, margin=self.pretrain_margin, seed=torch.initial_seed())
        return self._pstep

    def pretrain_Extractor(self, rng=None):
        """:289-348: pretrain_times + 1 steps over Extractor_generate batches (utils.py:548-613),
        margin loss relu(pretrain_margin - (query - false)).mean(), Adam; prints the reference's
        'Step: ...' line every pretrain_loss_every steps; then save_pretrain. Each step is one
        hipGraph replay (mmre.extractor_train.PretrainStep). rng: the batch generator's
        random.Random (the reference's module-level random is unseeded)."""
        import random
        from collections import deque
        from mmre.extractor_train import extractor_generate
        step = self._pretrain_step()
        losses = deque([], 100)
        batches = extractor_generate(self.train_tasks, self.rel2candidates, self.e1rel_e2, self.ent2id,
                                     self.pretrain_batch_size, self.pretrain_few, self.pretrain_subepoch,
                                     rng if rng is not None else random.Random())
        dev = self.device
        i = 0
        for data in batches:
            i += 1
            loss = step.replay({k: torch.as_tensor(v, device=dev) for k, v in data.items()})
            losses.append(float(loss))
            if i % self.pretrain_loss_every == 0:
                print("Step: %d, Feature Extractor Pretraining loss: %.2f" % (i, np.mean(losses)))
            if i > self.pretrain_times:
                break
        self.pretrain_losses = list(losses)
        self.save_pretrain()

    def _ranker(self):
        self.Extractor.eval()
        return ZSLRanker(self.Extractor, self.graph.ent_sym, self.graph.connections, self.graph.e1_degrees,
                         device=self.device)

    def _centroids(self, ranker, vecs_fn=None):
        """centroid_matrix (:353-383): the mean Extractor vector of every train relation's pairs
        (centroid_generate, utils.py:615-623), row rela2label[relation]; one encode launch
        (vecs_fn: the training-mode Extractor's vectors instead, dropout included)."""
        heads, tails, labels = [], [], []
        for rel, triples in self.train_tasks.items():
            heads += [self.ent2id[t[0]] for t in triples]
            tails += [self.ent2id[t[2]] for t in triples]
            labels += [self.rela2label[rel]] * len(triples)
        dev = self.device
        h, t, lab = (torch.as_tensor(x, dtype=torch.int64, device=dev) for x in (heads, tails, labels))
        if vecs_fn is not None:
            g = vecs_fn(h, t)
        else:
            g, _ = encode(ranker.pack, ranker.dim, ranker.ln_eps, ranker.left, h, ranker.right, t, want_g=True,
                          want_score=False)
        sums = torch.zeros((len(self.train_tasks), self.emb_dim), dtype=torch.float32, device=dev)
        sums.index_add_(0, lab, g)
        cnt = torch.bincount(lab, minlength=len(self.train_tasks)).clamp(min=1).to(torch.float32)
        return sums / cnt.unsqueeze(1)

    def train(self, generate_model=None):
        """:350-633. train() without a model is nn.Module.train() (mode switch)."""
        if generate_model is None or isinstance(generate_model, bool):
            return super().train(True if generate_model is None else generate_model)
        import random
        from mmre.gan import ZSLGANStep
        print("\n##START ADVERSARIAL TRAINING...")
        extractor_training = self.Extractor.training
        self.pretrain_Extractor()
        grad_list = ["generate_fc_layer.weight_orig", "generate_fc_layer.bias", "des_rel_map_layer1.weight_orig",
                     "des_rel_map_layer1.bias", "des_rel_map_layer2.weight_orig", "des_rel_map_layer2.bias",
                     "layer_norm.a_2", "layer_norm.b_2"]
        for name, param in generate_model.named_parameters():
            param.requires_grad = name in grad_list
        ranker = self._ranker()
        self.Extractor.train(extractor_training)
        vecs_fn = None
        if extractor_training:  # the reference's Extractor is still in training mode here: dropout vectors
            vecs_fn = self._pretrain_step().vectors
        self.centroid_matrix = self._centroids(ranker, vecs_fn)
        dev = self.device
        cls_table = generate_model.M3AEmodel.encode(self.des_tokens.to(dev), self.des_pad_masks.to(dev))
        self.gan_step = ZSLGANStep(generate_model.generator, self.Discriminator, cls_table, self.centroid_matrix,
                                   ranker, lr_G=self.lr_maximum, lr_D=self.lr_D, pretrain_margin=self.pretrain_margin,
                                   gan_batch_rela=self.gan_batch_rela, vecs_fn=vecs_fn)
        print("##LOADING TRAINING DATA")
        batches = train_generate_decription(self.train_tasks, self.rel2candidates, self.e1rel_e2, self.ent2id,
                                            self.rel2id, self.rela2label, self.G_batch_size, self.gan_batch_rela,
                                            rng=random.Random())
        gan_train(self.gan_step, batches, self.train_times, D_epoch=self.D_epoch, G_epoch=self.G_epoch,
                  loss_every=self.loss_every, device=dev)
        self.save(generate_model)
        return self.eval(generate_model, mode="test", meta=self.meta)

    # ---------------------------------------------------------------- evaluation
    def relation_vectors(self, generate_model, relations):
        """generate() of test_sample rows per relation with the fixed test noises (:662-667),
        all relations in one call (eval mode: every row depends on its own CLS and noise only)."""
        dev = self.device
        S = int(self.test_sample)
        ids = torch.as_tensor([self.rel2id[r] for r in relations], dtype=torch.int64)
        tok = self.des_tokens[ids].repeat_interleave(S, 0).to(dev)
        msk = self.des_pad_masks[ids].repeat_interleave(S, 0).to(dev)
        noise = self.test_noises.repeat(len(relations), 1)
        with torch.no_grad():
            out = generate_model.generate(tok, msk, noise)
        return out.view(len(relations), S, -1)

    def eval(self, generate_model=None, mode="test", meta=True, load_pretrain=False):
        """:635-745 -> (hits10, hits5, mrr); prints the reference's per-relation and final
        lines. eval() without a model is nn.Module.eval() (mode switch)."""
        if generate_model is None:
            return super().eval()
        if load_pretrain:
            self.load_pretrain()
            self.load(generate_model)
        generate_model.eval()
        self.Discriminator.eval()
        self.Extractor.eval()
        print("##EVALUATING ON %s DATA" % mode.upper())
        if not meta:
            raise MMREError("ZSLmodule.eval scores candidates only with meta=True (zsl_module.py:690-703)")
        test_candidates = _read_json(self.data_path + "/" + mode + "_candidates.json")
        rels = list(test_candidates.keys())
        vecs = self.relation_vectors(generate_model, rels)
        evaluator = ZSLEvaluator(self.Extractor, self.graph, device=self.device)
        return evaluator.eval(dict(zip(rels, vecs)), test_candidates, mode)

    # ---------------------------------------------------------------- checkpoints (:205-207, 747-755)
    def save(self, generate_model):
        os.makedirs(self.save_path, exist_ok=True)
        torch.save(generate_model.state_dict(), os.path.join(self.save_path, "Generator"))
        torch.save(self.Discriminator.state_dict(), os.path.join(self.save_path, "Discriminator"))

    def load(self, generate_model):
        generate_model.load_state_dict(torch.load(os.path.join(self.save_path, "Generator"),
                                                  map_location=self.device, weights_only=True))
        self.Discriminator.load_state_dict(torch.load(os.path.join(self.save_path, "Discriminator"),
                                                      map_location=self.device, weights_only=True))

    def save_pretrain(self):
        os.makedirs(self.save_path, exist_ok=True)
        torch.save(self.Extractor.state_dict(), os.path.join(self.save_path, "Extractor"))

    def load_pretrain(self):
        self.Extractor.load_state_dict(torch.load(os.path.join(self.save_path, "Extractor"),
                                                  map_location=self.device, weights_only=True))
