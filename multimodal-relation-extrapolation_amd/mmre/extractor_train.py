"""The ZSL Extractor in training mode and its pretraining step (pretrain_Extractor,
module/zsl_module.py:289-348), on the GPU.

Training-mode forward of one (e1, e2) row (zsl_module.py:47-110, submodule.py:254-258), dropout
p = 0.2 at three places:

    left  = tanh( sum_s gcn_w(dropout(emb[conn_l[s]])) / deg_l )
    ent   = tanh( cat(fc1(dropout_e(emb[e1])), fc2(dropout_e(emb[e2]))) )
    x     = reshape_layer( cat(left, ent, right) )
    g     = LayerNorm( dropout(proj2(relu(proj1(x)))) + x )

symbol_emb is frozen (:38), so the dropped neighbour sums and entity rows are constants of the
step, gathered per row by one HIP launch (mmre_extractor_train_inputs; gcn_w is linear, so it
is applied once to the sum: W sum_s x_s + max_nb b). The rest is an autograd chain whose every
product runs on the split-K GEMM (mmre.gemm.mm, csrc/gemm.hip) and whose SupportEncoder dropout
is mmre_dropout. Masks are a counter hash of a device (seed, offset) pair, so a step captured in
a hipGraph draws fresh masks at each replay.

`PretrainStep` is one pretraining step: the support / query / false rows of an
Extractor_generate batch (module/utils.py:548-613) through two Extractor calls -- the support
set is encoded once per call, with its own masks, exactly as the reference's two
`self.Extractor(...)` calls do (:318-323) -- the margin loss relu(margin - (query - false)).mean()
(:325-326), backward and torch's Adam (optim_E, lr_E; :183-186). Each batch shape is captured once
into a hipGraph and replayed.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ._lib import MMREError, call, ptr, require_cuda, stream_ptr
from .gemm import mm

DROPOUT_P = 0.2          # nn.Dropout(0.2) of the Extractor and its SupportEncoder (zsl_module.py:34-35, :43)
STREAM_SUPPORT_ENC = 3   # dropout streams 0-2: neighbour sums (left, right), entity rows


class DropoutRNG:
    """Device (seed, offset) pair behind every training-mode mask; `advance()` is an in-graph
    add, so each replay of a captured step draws new masks."""

    def __init__(self, seed: int, device):
        self.state = torch.tensor([int(seed) & 0x7FFFFFFFFFFFFFFF, 0], dtype=torch.int64, device=device)

    def advance(self, by: int = 1):
        self.state[1:].add_(by)


def train_inputs(emb, pairs, meta, p, rng=None, masks=None, check=True):
    """(nsum_left, nsum_right, e1, e2), each (B, d): the dropped constants of the forward.
    masks (tests): (nb_left (B, M, d), nb_right (B, M, d), ent (B, 2, d)) 0/1 uint8.
    check: validate the symbol ids on the host (a device sync; off inside a graph capture,
    where the ids come from the device tables themselves)."""
    lc, _, rc, _ = meta
    B, d = int(pairs.shape[0]), int(emb.shape[1])
    M = int(lc.shape[1])
    require_cuda(emb, pairs, lc, rc)
    if lc.shape != (B, M, 2) or rc.shape != (B, M, 2):
        raise MMREError("connections must be (rows, max_neighbor, 2)")
    n_sym = int(emb.shape[0])
    if check and not torch.cuda.is_current_stream_capturing():
        for ids in (pairs, lc[:, :, 1], rc[:, :, 1]):
            if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= n_sym):
                raise MMREError("symbol id outside symbol_emb")
    dev = emb.device
    out = [torch.empty((B, d), dtype=torch.float32, device=dev) for _ in range(4)]
    if masks is not None:
        m = [x.to(device=dev, dtype=torch.uint8).contiguous() for x in masks]
        if m[0].shape != (B, M, d) or m[1].shape != (B, M, d) or m[2].shape != (B, 2, d):
            raise MMREError("masks: (B, M, d), (B, M, d), (B, 2, d)")
    else:
        m = [None, None, None]
        if rng is None:
            raise MMREError("train_inputs needs a DropoutRNG or explicit masks")
    call("mmre_extractor_train_inputs", d, ptr(emb.detach().contiguous()), ptr(pairs.contiguous().long()),
         ptr(lc.contiguous().long()), ptr(rc.contiguous().long()), M, B, float(p),
         ptr(rng.state) if rng is not None else None, ptr(m[0]), ptr(m[1]), ptr(m[2]), *[ptr(o) for o in out],
         stream_ptr(dev))
    return out


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, state, stream_id, mask):
        x = x.contiguous()
        y = torch.empty_like(x)
        if mask is None:
            mask = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
            call("mmre_dropout", ptr(x), ptr(y), ptr(mask), x.numel(), float(p), ptr(state), int(stream_id),
                 stream_ptr(x.device))
        else:
            y = x * (mask.to(x.dtype) * (1.0 / (1.0 - p)))
        ctx.save_for_backward(mask)
        ctx.scale = 1.0 / (1.0 - p)
        return y

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        return g * (mask.to(g.dtype) * ctx.scale), None, None, None, None


def dropout(x, p, rng, stream_id, mask=None):
    if p == 0.0:
        return x
    return _Dropout.apply(x, float(p), None if rng is None else rng.state, int(stream_id), mask)


def train_forward(ex, pairs, meta, p=DROPOUT_P, rng=None, masks=None, check=True):
    """query_g (B, d) of the Extractor in training mode, differentiable w.r.t. its parameters.
    masks (tests): (nb_left, nb_right, ent, support_encoder (B, d)) 0/1. Rows of one call draw
    independent masks; a second call draws the same masks unless rng.advance() ran between."""
    emb = ex.symbol_emb.weight
    lc, ld, rc, rd = meta
    nl, nr, e1, e2 = train_inputs(emb, pairs, meta, p, rng, None if masks is None else masks[:3], check=check)
    M = float(lc.shape[1])
    W = ex.gcn_w
    gb = W.bias * M                                    # sum over the max_nb slots of the per-slot bias
    left = torch.tanh(mm(nl, W.weight.t(), gb) / ld.unsqueeze(1))
    right = torch.tanh(mm(nr, W.weight.t(), gb) / rd.unsqueeze(1))
    ent = torch.tanh(torch.cat((mm(e1, ex.fc1.weight.t(), ex.fc1.bias), mm(e2, ex.fc2.weight.t(), ex.fc2.bias)), -1))
    x = mm(torch.cat((left, ent, right), -1), ex.reshape_layer.weight.t(), ex.reshape_layer.bias)
    se = ex.support_encoder
    h = F.relu(mm(x, se.proj1.weight.t(), se.proj1.bias))
    y = dropout(mm(h, se.proj2.weight.t(), se.proj2.bias), p, rng, STREAM_SUPPORT_ENC,
                None if masks is None else masks[3].to(device=x.device, dtype=torch.uint8))
    return F.layer_norm(y + x, (y.shape[1],), se.layer_norm.weight, se.layer_norm.bias, se.layer_norm.eps)


class PretrainStep:
    """pretrain_Extractor's step (zsl_module.py:296-344) for an Extractor `ex` over the device
    graph tables (ent_sym (E,), connections (E, M, 2), degrees (E,) float: ZSLGraph). Rows are
    entity ids; symbols and neighbour lists are gathered on the device (get_meta, :265-287)."""

    def __init__(self, ex, ent_sym, conn, deg, lr=1e-4, margin=5.0, seed=0, p=None):
        self.ex = ex
        dev = ex.symbol_emb.weight.device
        self.device = dev
        self.ent_sym, self.conn, self.deg = ent_sym.to(dev), conn.to(dev), deg.to(dev).float()
        self.margin = float(margin)
        self.p = p
        self.params = [q for q in ex.parameters() if q.requires_grad]
        self.optim = torch.optim.Adam(self.params, lr=lr, capturable=True)
        self.rng = DropoutRNG(seed, dev)
        self._graphs = {}
        self._static = {}
        self.keep_grads = False

    def _p(self):
        return (DROPOUT_P if self.ex.training else 0.0) if self.p is None else float(self.p)

    def rows(self, heads, tails):
        """(pairs, meta) of entity-id rows: ZSLmodule.get_meta + the symbol pair."""
        pairs = torch.stack((self.ent_sym[heads], self.ent_sym[tails]), 1)
        return pairs, (self.conn[heads], self.deg[heads], self.conn[tails], self.deg[tails])

    def loss(self, s_h, s_t, q_h, q_t, f_h, f_t, masks=None):
        """margin loss of one batch; rows are encoded as [support | query | support | false]
        (two Extractor calls, each with its own support encoding)."""
        S, Q = int(s_h.shape[0]), int(q_h.shape[0])
        heads = torch.cat((s_h, q_h, s_h, f_h))
        tails = torch.cat((s_t, q_t, s_t, f_t))
        pairs, meta = self.rows(heads, tails)
        g = train_forward(self.ex, pairs, meta, self._p(), self.rng, masks, check=False)
        s1 = g[:S].mean(0)
        s2 = g[S + Q:2 * S + Q].mean(0)
        q_scores = mm(g[S:S + Q], s1.unsqueeze(1)).squeeze(1)
        f_scores = mm(g[2 * S + Q:], s2.unsqueeze(1)).squeeze(1)
        return F.relu(self.margin - (q_scores - f_scores)).mean()

    def vectors(self, heads, tails):
        """Extractor vectors of entity-id rows in the Extractor's current mode, no gradient
        (the GAN loop's real / false / centroid vectors, zsl_module.py:371-383, 430-440);
        in training mode each call draws its own masks."""
        pairs, meta = self.rows(heads, tails)
        with torch.no_grad():
            g = train_forward(self.ex, pairs, meta, self._p(), self.rng, check=False)
        self.rng.advance()
        return g

    def step(self, s_h, s_t, q_h, q_t, f_h, f_t, masks=None):
        loss = self.loss(s_h, s_t, q_h, q_t, f_h, f_t, masks)
        self.optim.zero_grad(set_to_none=False)
        loss.backward()
        if self.keep_grads:
            self.grads = [None if q.grad is None else q.grad.detach().clone() for q in self.params]
        self.optim.step()
        self.rng.advance()
        return loss.detach()

    # ------------------------------------------------------------ hipGraph replay
    def replay(self, batch):
        """batch: dict of device int64 entity ids s_h, s_t, q_h, q_t, f_h, f_t. The first call
        per shape runs eagerly (the warm-up a capture needs) and captures; later calls replay.
        Returns the loss (the graph's static output, overwritten by the next replay)."""
        keys = ("s_h", "s_t", "q_h", "q_t", "f_h", "f_t")
        n_ent = int(self.ent_sym.shape[0])
        for k in keys:
            v = batch[k]
            if v.numel() and (int(v.min()) < 0 or int(v.max()) >= n_ent):
                raise MMREError(f"pretrain batch {k}: entity id outside the graph")
        # the dropout rate is baked into a capture: the key holds it (the Extractor's mode may change)
        shape = (int(batch["s_h"].shape[0]), int(batch["q_h"].shape[0]), int(batch["f_h"].shape[0]), self._p())
        if shape not in self._static:
            self._static[shape] = {k: torch.zeros_like(batch[k]) for k in keys}
        b = self._static[shape]
        for k in keys:
            b[k].copy_(batch[k], non_blocking=True)
        if shape in self._graphs:
            g, out = self._graphs[shape]
            g.replay()
            return out
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            first = self.step(*(b[k] for k in keys))
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self.step(*(b[k] for k in keys))
        self._graphs[shape] = (graph, out)
        return first


def extractor_generate(train_tasks, rel2candidates, e1rel_e2, ent2id, batch_size, few, sub_epoch, rng):
    """Extractor_generate (module/utils.py:548-613) as entity-id arrays. Per batch: one train
    relation drawn with probability proportional to min(#candidates, 1000) (0 when <= 20
    candidates; random_pick, utils.py:238-244), then sub_epoch times: shuffle its triples, the
    first `few` are support, `batch_size` queries from the rest (with replacement when fewer),
    one false tail per query from the relation's candidates (in ent2id, not a known tail of
    (head, rel), not the true tail). Yields dict(s_h, s_t, q_h, q_t, f_h, f_t) int64 arrays.
    rng: random.Random (the reference draws from the unseeded module-level random)."""
    pool = list(train_tasks.keys())
    weights = [0 if len(rel2candidates[k]) <= 20 else min(len(rel2candidates[k]), 1000) for k in pool]
    total = float(sum(weights))
    if total <= 0:
        raise MMREError("Extractor_generate: no train relation has more than 20 candidates")
    prob = [w / total for w in weights]
    while True:
        out = {k: [] for k in ("s_h", "s_t", "q_h", "q_t", "f_h", "f_t")}
        x, cum, query = rng.uniform(0, 1), 0.0, pool[-1]
        for item, pr in zip(pool, prob):   # random_pick
            cum += pr
            if x < cum:
                query = item
                break
        cands = rel2candidates[query]
        for _ in range(sub_epoch):
            triples = train_tasks[query]
            rng.shuffle(triples)
            support = triples[:few]
            out["s_h"] += [ent2id[t[0]] for t in support]
            out["s_t"] += [ent2id[t[2]] for t in support]
            rest = triples[few:]
            if not rest:
                continue
            qs = [rng.choice(rest) for _ in range(batch_size)] if len(rest) < batch_size else rng.sample(rest, batch_size)
            out["q_h"] += [ent2id[t[0]] for t in qs]
            out["q_t"] += [ent2id[t[2]] for t in qs]
            for h, r, t in qs:
                while True:
                    noise = rng.choice(cands)
                    if noise in ent2id and noise not in e1rel_e2[h + r] and noise != t:
                        break
                out["f_h"].append(ent2id[h])
                out["f_t"].append(ent2id[noise])
        yield {k: np.asarray(v, np.int64) for k, v in out.items()}
