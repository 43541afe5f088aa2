"""ZSL Extractor + cosine ranking on the GPU (csrc/extractor.hip).

The Extractor of ZSLmodule (module/zsl_module.py:17-110) maps a (head, tail) entity pair to a
d-dim vector; ZSLmodule.eval (zsl_module.py:635-745) ranks each query's candidate tails by the
mean cosine similarity of that vector with the relation's generated vectors. Here:

  * `pack_weights` lays the Extractor's nn.Linear weights out in MFMA lane order once;
  * `node_tables` computes, per entity, the two halves of reshape_layer's output
    (neighbour encoder + entity encoder folded through the linear reshape_layer), so a
    candidate row costs only the SupportEncoder;
  * `encode` runs SupportEncoder + LayerNorm (+ cosine against a target) for any list of
    (left node, right node) rows, 16 rows per wave on v_mfma_f32_16x16x4_f32;
  * `ZSLRanker.rank` is one ZSL evaluation: every query's candidate list scored and ranked in
    one launch sequence, ranks = 1 + #(score > score[true]) (zsl_module.py:705-706).
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import MMREError, call, lib, ptr, require_cuda, stream_ptr

SUPPORTED_DIMS = (64, 100, 128, 200, 256)


def _c(t):
    return t.detach().contiguous().float()


def pack_weights(ex) -> torch.Tensor:
    """ex: a module with the reference Extractor's parameter names (gcn_w, fc1, fc2,
    reshape_layer, support_encoder.{proj1, proj2, layer_norm})."""
    d = int(ex.embed_dim)
    if d not in SUPPORTED_DIMS:
        raise MMREError(f"Extractor embed_dim {d} not built (supported: {SUPPORTED_DIMS})")
    dev = ex.gcn_w.weight.device
    n = int(lib().mmre_extractor_pack_size(d))
    pack = torch.empty(n, dtype=torch.float32, device=dev)
    se = ex.support_encoder
    ws = [ex.gcn_w.weight, ex.gcn_w.bias, ex.fc1.weight, ex.fc1.bias, ex.fc2.weight, ex.fc2.bias,
          ex.reshape_layer.weight, ex.reshape_layer.bias, se.proj1.weight, se.proj1.bias, se.proj2.weight,
          se.proj2.bias, se.layer_norm.weight, se.layer_norm.bias]
    ws = [_c(w) for w in ws]
    require_cuda(*ws)
    call("mmre_extractor_pack", d, *[ptr(w) for w in ws], ptr(pack), stream_ptr(dev))
    return pack


def node_tables(pack, dim: int, sym_emb, node_sym, conn, deg, want_left=True, want_right=True):
    """(left, right) per-node tables (n, dim) (either may be None)."""
    require_cuda(pack, sym_emb, node_sym, conn, deg)
    n = int(node_sym.shape[0])
    dev = sym_emb.device
    if conn.dim() != 3 or conn.shape[0] != n or conn.shape[2] != 2 or deg.shape[0] != n:
        raise MMREError("connections must be (n, max_neighbor, 2) and degrees (n,)")
    left = torch.empty((n, dim), dtype=torch.float32, device=dev) if want_left else None
    right = torch.empty((n, dim), dtype=torch.float32, device=dev) if want_right else None
    if n == 0:
        return left, right
    call("mmre_extractor_nodes", dim, ptr(pack), ptr(_c(sym_emb)), ptr(node_sym.contiguous().long()),
         ptr(conn.contiguous().long()), int(conn.shape[1]), ptr(deg.contiguous().float()), n, ptr(left),
         ptr(right), stream_ptr(dev))
    return left, right


def encode(pack, dim: int, ln_eps: float, left, li, right, ri, targets=None, row_target=None, normalize=True,
           want_g=False, want_score=True):
    """SupportEncoder(left[li] + right[ri]) -> (g (n, dim) or None, score (n,) or None)."""
    require_cuda(pack, left, li, right, ri, targets, row_target)
    n = int(li.shape[0])
    dev = left.device
    g = torch.empty((n, dim), dtype=torch.float32, device=dev) if want_g else None
    s = torch.empty(n, dtype=torch.float32, device=dev) if want_score else None
    if n == 0:
        return g, s
    if want_score and targets is None:
        raise MMREError("scores need targets")
    call("mmre_extractor_encode", dim, ptr(pack), float(ln_eps), ptr(left), ptr(li.contiguous().long()), ptr(right),
         ptr(ri.contiguous().long()), n, ptr(None if targets is None else _c(targets)),
         ptr(None if row_target is None else row_target.contiguous().long()), int(bool(normalize)), ptr(g), ptr(s),
         stream_ptr(dev))
    return g, s


def targets(vecs, normalize=True):
    """vecs (T, S, d) -> (T, d) mean over S of the (L2-normalised) rows."""
    require_cuda(vecs)
    T, S, d = (int(x) for x in vecs.shape)
    out = torch.empty((T, d), dtype=torch.float32, device=vecs.device)
    call("mmre_extractor_targets", ptr(_c(vecs)), T, S, d, int(bool(normalize)), ptr(out), stream_ptr(vecs.device))
    return out


def rank_desc(scores, off):
    """rank of the first entry of each CSR list: 1 + #(score > score[first])."""
    require_cuda(scores, off)
    q = int(off.shape[0]) - 1
    rank = torch.empty(q, dtype=torch.int32, device=scores.device)
    if q > 0:
        call("mmre_rank_desc", ptr(scores.contiguous()), ptr(off.contiguous().long()), q, ptr(rank),
             stream_ptr(scores.device))
    return rank


class ZSLRanker:
    """Fused ZSL evaluation over a fixed entity graph (ZSLmodule.eval, zsl_module.py:666-706).

    extractor: the Extractor module (its symbol_emb holds symbol2vec, load_embed :208-232);
    ent_sym (E,): symbol id of each entity id; connections (E, max_neighbor, 2) and
    degrees (E,) as built by build_connection (:233-263)."""

    def __init__(self, extractor, ent_sym, connections, degrees, device=None):
        dev = torch.device(device) if device is not None else extractor.gcn_w.weight.device
        self.dim = int(extractor.embed_dim)
        self.ln_eps = float(extractor.support_encoder.layer_norm.eps)
        to = lambda a, dt: torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a).to(dev, dt).contiguous()
        self.ent_sym = to(ent_sym, torch.int64)
        self.conn = to(connections, torch.int64)
        self.deg = to(degrees, torch.float32)
        n_sym = int(extractor.symbol_emb.weight.shape[0])
        _check_ids(self.ent_sym, n_sym, "entity symbol ids")
        _check_ids(self.conn[:, :, 1], n_sym, "neighbour symbol ids")
        self.extractor = extractor
        self.refresh()

    def refresh(self):
        """Re-pack weights and rebuild the per-entity tables (after weights/embeddings change)."""
        ex = self.extractor
        self.pack = pack_weights(ex)
        self.left, self.right = node_tables(self.pack, self.dim, ex.symbol_emb.weight, self.ent_sym, self.conn,
                                            self.deg)

    def scores(self, cand_head, cand_tail, row_set, rel_targets):
        _, s = encode(self.pack, self.dim, self.ln_eps, self.left, cand_head, self.right, cand_tail,
                      targets=rel_targets, row_target=row_set, normalize=True)
        return s

    def rank(self, cand_head, cand_tail, off, rel_vecs, query_set, return_scores=False):
        """cand_head / cand_tail (N,) entity ids, the true pair first in each query's CSR slice
        off (Q+1,); rel_vecs (T, S, d) generated relation vectors; query_set (Q,) -> row of
        rel_vecs each query uses. Returns int32 ranks (Q,)."""
        dev = self.left.device
        off = off.to(dev).long()
        counts = off[1:] - off[:-1]
        row_set = torch.repeat_interleave(query_set.to(dev).long(), counts)
        t = targets(rel_vecs.to(dev), normalize=True)
        s = self.scores(cand_head.to(dev), cand_tail.to(dev), row_set, t)
        r = rank_desc(s, off)
        return (r, s) if return_scores else r


def _check_ids(ids, n_sym, what):
    if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= n_sym):
        raise MMREError(f"{what} out of range [0, {n_sym})")


def support_encode(se, x):
    """SupportEncoder.forward (submodule.py:254-258) for x (n, d) in eval mode: the encode
    kernel with left = x, right = 0 and the neighbour/entity weights unused."""
    if se.training:
        raise MMREError("SupportEncoder runs in eval mode only on this path (dropout is training-only)")
    require_cuda(x)
    d = int(x.shape[-1])
    if 2 * d != se.proj1.out_features:
        raise MMREError("SupportEncoder d_inner must be 2 * d_model (the Extractor's shape)")
    if d not in SUPPORTED_DIMS:
        raise MMREError(f"d {d} not built (supported: {SUPPORTED_DIMS})")
    dev = x.device
    z = lambda *s: torch.zeros(s, dtype=torch.float32, device=dev)
    h = d // 2
    ws = [z(h, d), z(h), z(h, d), z(h), z(h, d), z(h), z(d, 2 * d), z(d), _c(se.proj1.weight), _c(se.proj1.bias),
          _c(se.proj2.weight), _c(se.proj2.bias), _c(se.layer_norm.weight), _c(se.layer_norm.bias)]
    pack = torch.empty(int(lib().mmre_extractor_pack_size(d)), dtype=torch.float32, device=dev)
    call("mmre_extractor_pack", d, *[ptr(w) for w in ws], ptr(pack), stream_ptr(dev))
    x2 = _c(x.reshape(-1, d))
    n = x2.shape[0]
    idx = torch.arange(n, device=dev)
    g, _ = encode(pack, d, float(se.layer_norm.eps), x2, idx, z(1, d), torch.zeros_like(idx), want_g=True,
                  want_score=False)
    return g.reshape(x.shape)
