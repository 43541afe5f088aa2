"""Link prediction engine: the fused all-entity sweep + rank epilogue on the GPU.

One `LinkSweep.run` call replaces the whole per-query loop of the reference
Tester (OpenKE/openke/config/Tester.py:70-91): getHeadBatch/getTailBatch
(Test.h:36-53) -> model.predict (a D2H copy of E scores per query) ->
testHead/testTail (Test.h:65-192). Here every head- and tail-batch query of the
evaluation is scored against every entity in one launch sequence, and only the
integer rank counts come back.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

MODEL_IDS = {"transe": 0, "transe_l2": 1, "distmult": 2, "complex": 3, "rotate": 4}
HEAD, TAIL = 0, 1
METRIC_NAMES = ["mrr", "mr", "hit10", "hit3", "hit1"]
GROUPS = ["filter", "raw", "filter_tc", "raw_tc"]


@dataclass
class ScoreSpec:
    """How a model scores: which kernel, which tables, and predict's transform."""
    model: str                      # key of MODEL_IDS
    ent: torch.Tensor               # (E, d) or RotatE (E, 2d); ComplEx: real part
    rel: torch.Tensor               # (R, d); ComplEx: real part
    dim: int
    ent_im: torch.Tensor | None = None
    rel_im: torch.Tensor | None = None
    norm_flag: bool = False
    pred_kind: int = 0              # 0 s, 1 m-(m-s), 2 -s, 3 -(m-s)
    margin: float = 0.0
    phase_denom: float = 0.0        # RotatE


def rotate_phase_denom(margin: float, epsilon: float, dim: int) -> float:
    """RotatE.py:51 ``r / (rel_embedding_range.item() / pi)``: torch evaluates the python-float /
    float32-tensor quotient as ``reciprocal(pi) * range`` in float32."""
    rng = np.float32((margin + epsilon) / dim)
    pi = np.float32(3.14159265358979323846)
    return float(np.float32(np.float32(np.float32(1.0) / pi) * rng))


class FilterIndex:
    """Known-triple index (train + valid + test, Reader.h:201-226) for filtered ranks, and the
    per-relation type constraints (type_constrain.txt, Reader.h:266-317), as device CSR lists /
    bitsets for the sweep's epilogue."""

    def __init__(self, h, r, t, n_ent: int, n_rel: int, type_heads=None, type_tails=None):
        a = np.unique(np.stack([np.asarray(h, np.int64), np.asarray(r, np.int64), np.asarray(t, np.int64)], 1),
                      axis=0)
        self.n_ent, self.n_rel = int(n_ent), int(n_rel)
        # tail filter: (h, r) -> tails ; head filter: (r, t) -> heads
        self._hr_key = a[:, 0] * n_rel + a[:, 1]
        o = np.lexsort((a[:, 2], self._hr_key))
        self._hr_key, self._hr_val = self._hr_key[o], a[o, 2]
        self._rt_key = a[:, 1] * n_ent + a[:, 2]
        o = np.lexsort((a[:, 0], self._rt_key))
        self._rt_key, self._rt_val = self._rt_key[o], a[o, 0]
        self.type_heads, self.type_tails = type_heads, type_tails

    @staticmethod
    def _gather(keys, vals, qkeys):
        s = np.searchsorted(keys, qkeys, "left")
        e = np.searchsorted(keys, qkeys, "right")
        ln = e - s
        off = np.zeros(len(qkeys) + 1, np.int64)
        np.cumsum(ln, out=off[1:])
        idx = np.repeat(s - off[:-1], ln) + np.arange(off[-1])
        return off, vals[idx].astype(np.int32)

    def filters(self, qh, qr, qt, qmode):
        qh, qr, qt, qmode = (np.asarray(x, np.int64) for x in (qh, qr, qt, qmode))
        n = len(qh)
        off = np.zeros(n + 1, np.int64)
        head = qmode == HEAD
        lens = np.zeros(n, np.int64)
        per = [None] * 2
        if head.any():
            per[0] = self._gather(self._rt_key, self._rt_val, qr[head] * self.n_ent + qt[head])
            lens[head] = np.diff(per[0][0])
        if (~head).any():
            per[1] = self._gather(self._hr_key, self._hr_val, qh[~head] * self.n_rel + qr[~head])
            lens[~head] = np.diff(per[1][0])
        np.cumsum(lens, out=off[1:])
        ids = np.empty(off[-1], np.int32)
        # scatter each group's lists into query order
        for g, mask in ((0, head), (1, ~head)):
            if per[g] is None:
                continue
            goff, gids = per[g]
            qi = np.nonzero(mask)[0]
            dst = np.repeat(off[qi] - goff[:-1], np.diff(goff)) + np.arange(goff[-1])
            ids[dst] = gids
        return off, ids

    def groups(self, qh, qr, qt, qmode, max_group: int = 64, entity_range=None):
        """Filter groups: queries with the same (mode, r, anchor) share their known-entity
        list (Test.h:85 `_find` looks up (r, t) for head_batch, (h, r) for tail_batch).
        Groups larger than `max_group` queries are split (one wave of the count kernel per
        group). Returns (grp_qoff int64 [G+1], grp_q int32 [Q], off int64 [G+1], ids int32,
        entry_q int32): the query partition, one CSR list per group and, per listed entity,
        the group member whose query vector scores it -- for mmre_link_truth_grouped.
        entity_range (e0, e1): keep only listed entities in [e0, e1) -- the filter correction of
        a rank that sweeps that slice of the table (entity-sharded evaluation)."""
        qh, qr, qt, qmode = (np.asarray(x, np.int64) for x in (qh, qr, qt, qmode))
        anchor = np.where(qmode == HEAD, qt, qh)
        key = (qmode * self.n_rel + qr) * self.n_ent + anchor
        _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        grp_q = np.argsort(inv, kind="stable").astype(np.int32)
        # split each key's run of queries into pieces of <= max_group
        starts = np.zeros(len(cnt), np.int64)
        np.cumsum(cnt[:-1], out=starts[1:])
        pieces = (cnt + max_group - 1) // max_group
        piece_key = np.repeat(np.arange(len(cnt)), pieces)
        piece_idx = np.arange(len(piece_key)) - np.repeat(np.cumsum(pieces) - pieces, pieces)
        grp_qoff = np.empty(len(piece_key) + 1, np.int64)
        grp_qoff[:-1] = starts[piece_key] + piece_idx * max_group
        grp_qoff[-1] = len(grp_q)
        first = grp_q[grp_qoff[:-1]]
        off, ids = self.filters(qh[first], qr[first], qt[first], qmode[first])
        entry_q = np.repeat(first, np.diff(off)).astype(np.int32)
        if entity_range is not None:
            e0, e1 = entity_range
            keep = (ids >= e0) & (ids < e1)
            kept = np.concatenate([[0], np.cumsum(keep, dtype=np.int64)])[off]  # new CSR offsets
            off, ids, entry_q = kept, ids[keep], entry_q[keep]
        return grp_qoff, grp_q, off, ids, entry_q

    def type_masks(self):
        if self.type_heads is None:
            return None
        words = (self.n_ent + 31) // 32
        out = []
        for lists in (self.type_heads, self.type_tails):
            m = np.zeros((self.n_rel, words * 32), np.uint8)
            for r, ids in enumerate(lists):
                ids = np.asarray(ids, np.int64)
                ids = ids[(ids >= 0) & (ids < self.n_ent)]
                m[r, ids] = 1
            w = (m.reshape(self.n_rel, words, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)).sum(-1)
            out.append(np.ascontiguousarray(w.astype(np.uint32)))
        return out


class LinkSweep:
    """Device-resident link-prediction evaluator for one model snapshot."""

    def __init__(self, spec: ScoreSpec):
        self.spec = spec
        self.model_id = MODEL_IDS[spec.model]
        dev = spec.ent.device
        _lib.require_cuda(spec.ent, spec.rel, spec.ent_im, spec.rel_im)
        self.device = dev
        self.n_ent = int(spec.ent.shape[0])
        self.n_rel = int(spec.rel.shape[0])
        L = _lib.lib()
        self.K = int(L.mmre_link_k(self.model_id, spec.dim))
        self.e_pad = int(L.mmre_link_pad(self.n_ent))
        self._ent = spec.ent.detach().contiguous().float()
        self._rel = spec.rel.detach().contiguous().float()
        self._ent_im = None if spec.ent_im is None else spec.ent_im.detach().contiguous().float()
        self._rel_im = None if spec.rel_im is None else spec.rel_im.detach().contiguous().float()
        self.ent_km = torch.empty((self.K, self.e_pad), dtype=torch.float32, device=dev)
        self.ent_rows = torch.empty((self.n_ent, self.K), dtype=torch.float32, device=dev)
        self.rel_work = torch.empty((self.n_rel, spec.dim), dtype=torch.float32, device=dev)
        self.prepared = False
        # TransE L1 count-only sweeps through the integer filter (mmre_link_sweep_l1q);
        # MMRE_L1_FILTER=0 keeps the f32 sweep (A/B measurements)
        self.l1_filter = os.environ.get("MMRE_L1_FILTER", "1") != "0"
        # DistMult / ComplEx count-only sweeps without type constraints through the split-bf16
        # MFMA filter (mmre_link_sweep_bf3); MMRE_MFMA_FILTER=0 keeps the f32 MFMA sweep
        self.mfma_filter = os.environ.get("MMRE_MFMA_FILTER", "1") != "0"
        # count-only TransE L1 runs with filter groups as ONE call (mmre_link_evaluate_l1q, seven
        # launches instead of thirteen); MMRE_FUSED_EVAL=0 keeps the separate entry points
        self.fused_eval = os.environ.get("MMRE_FUSED_EVAL", "1") != "0"
        # DistMult count-only sweeps split the raw rows (mmre_link_sweep_bf3_rows); "0" keeps the
        # prepared k-major / row-major copies (A/B; read per instance: tests switch it)
        self.bf3_raw = os.environ.get("MMRE_BF3_RAW", "1") != "0"

    def prepare_entities(self):
        s = self.spec
        call("mmre_link_prepare_entities", self.model_id, int(bool(s.norm_flag)), ptr(self._ent), ptr(self._ent_im),
             self.n_ent, s.dim, ptr(self.ent_km), self.e_pad, ptr(self.ent_rows), stream_ptr(self.device))
        self.prepared = True

    def alloc_queries(self, n_query: int):
        q_pad = int(_lib.lib().mmre_link_pad(n_query))
        dev = self.device
        return dict(q_km=torch.empty((self.K, q_pad), dtype=torch.float32, device=dev),
                    q_rows=torch.empty((n_query, self.K), dtype=torch.float32, device=dev),
                    q_true=torch.empty(q_pad, dtype=torch.int32, device=dev),
                    counts=torch.empty((4, n_query), dtype=torch.int32, device=dev),
                    truth=torch.empty(n_query, dtype=torch.float32, device=dev), q_pad=q_pad)

    def run(self, qh, qr, qt, qmode, filt=None, type_masks=None, return_scores=False, buffers=None,
            prepare=True, sweep_events=None, q_rows=True, entity_range=None, undecided_q=None):
        """qh/qr/qt int64 and qmode int8 device tensors. filt: per-query CSR (off int64, ids int32)
        or filter groups (grp_qoff, grp_q, off, ids, entry_q), see FilterIndex.groups.
        sweep_events: optional (start, end) torch.cuda.Event pair recorded around the sweep kernel alone
        (on the stream the kernels are launched on). q_rows=False: no row-major query copy (the
        per-query truth/filter kernel then gathers the query vectors from the k-major plane).
        entity_range (e0, e1), e0 a multiple of 128: sweep only those entities (filt restricted
        to them: FilterIndex.groups(..., entity_range)); summing counts over a partition of the
        table gives the whole-table counts (mmre_link_sweep_range).
        undecided_q: optional (Q,) int32 device tensor receiving, per query, the pairs the L1
        filter rescored (fused TransE L1 runs only; the sharding's cost calibration).
        Returns dict(counts=(4, Q) int32 [raw, filt, raw_tc, filt_tc], truth=(Q,), scores=(Q, E)|None)."""
        s = self.spec
        n = int(qh.shape[0])
        if n > 0 and self._fusable(filt, type_masks, return_scores, prepare, sweep_events, q_rows):
            return self._run_fused(qh, qr, qt, qmode, filt, buffers, entity_range, undecided_q)
        if undecided_q is not None:
            raise ValueError("undecided_q: only the fused TransE L1 evaluation counts undecided pairs per query")
        if n == 0:  # e.g. a rank that owns no test relation (world > #relations): nothing to sweep
            if sweep_events is not None:  # keep the caller's timing events valid (an empty interval)
                sweep_events[0].record()
                sweep_events[1].record()
            z = torch.empty((4, 0), dtype=torch.int32, device=self.device)
            return dict(counts=z, truth=torch.empty(0, dtype=torch.float32, device=self.device),
                        scores=torch.empty((0, self.n_ent), dtype=torch.float32, device=self.device)
                        if return_scores else None)
        l1q = (self.model_id == MODEL_IDS["transe"] and not return_scores and q_rows and self.l1_filter)
        bf3 = (self.model_id in (MODEL_IDS["distmult"], MODEL_IDS["complex"]) and not return_scores and q_rows
               and type_masks is None and self.mfma_filter)
        # DistMult count-only with filter groups and K = d: the raw table IS the row-major copy, so no
        # prepared copies are written (mmre_link_sweep_bf3_rows splits the raw rows; C5: 2 GB of
        # re-laid-out writes per evaluation gone); MMRE_BF3_RAW=0 keeps the prepared path (A/B)
        raw = (bf3 and self.model_id == MODEL_IDS["distmult"] and self.K == s.dim and filt is not None
               and len(filt) == 5 and self._ent.data_ptr() % 16 == 0 and self.bf3_raw)
        ent_rows = self._ent if raw else self.ent_rows
        if not raw and (prepare or not self.prepared):
            self.prepare_entities()
        b = buffers if buffers is not None else self.alloc_queries(n)
        st = stream_ptr(self.device)
        qrow = b["q_rows"] if q_rows else None   # None: truth kernel reads the k-major plane
        call("mmre_link_prepare_queries", self.model_id, int(bool(s.norm_flag)), ptr(ent_rows), ptr(self._rel),
             ptr(self._rel_im), self.n_ent, self.n_rel, s.dim, float(s.phase_denom), ptr(qh), ptr(qr), ptr(qt),
             ptr(qmode), n, ptr(b["q_km"]), b["q_pad"], ptr(b["q_true"]), ptr(self.rel_work), ptr(qrow), st)
        scores = None
        if return_scores:
            scores = torch.empty((n, self.n_ent), dtype=torch.float32, device=self.device)
        th, tt = (None, None) if type_masks is None else type_masks
        if filt is not None and len(filt) == 5 and q_rows:   # filter groups (FilterIndex.groups)
            gqo, gq, off, ids, entry_q = filt
            n_entries = int(ids.shape[0])
            lv = b.get("list_scores")
            if lv is None or lv.shape[0] < n_entries:
                lv = b["list_scores"] = torch.empty(max(n_entries, 1), dtype=torch.float32, device=self.device)
            call("mmre_link_truth_grouped", self.model_id, int(s.pred_kind), float(s.margin), ptr(ent_rows),
                 self.n_ent, ptr(qrow), ptr(b["q_true"]), ptr(qr), ptr(qmode), n, s.dim, ptr(gqo), ptr(gq),
                 int(gqo.shape[0]) - 1, ptr(off), ptr(ids), ptr(entry_q), n_entries, ptr(th), ptr(tt), ptr(lv),
                 ptr(b["counts"]), ptr(b["truth"]), st)
        else:
            if filt is not None and len(filt) == 5:   # groups -> per-query CSR is not derivable here
                raise ValueError("filter groups need q_rows=True")
            off, ids = (None, None) if filt is None else filt
            call("mmre_link_truth", self.model_id, int(s.pred_kind), float(s.margin), ptr(self.ent_km), self.n_ent,
                 self.e_pad, ptr(self.ent_rows), ptr(b["q_km"]), ptr(b["q_true"]), ptr(qr), ptr(qmode), n,
                 b["q_pad"], s.dim, ptr(off), ptr(ids), ptr(th), ptr(tt), ptr(b["counts"]), ptr(b["truth"]), st)
        if l1q:
            need = int(_lib.lib().mmre_link_l1q_workspace(s.dim, self.e_pad, b["q_pad"]))
            wk = b.get("l1q_work")
            if wk is None or wk.numel() < need:
                wk = b["l1q_work"] = torch.empty(need, dtype=torch.uint8, device=self.device)
        if bf3:
            need = int(_lib.lib().mmre_link_bf3_workspace(self.model_id, s.dim, self.e_pad, b["q_pad"]))
            wk = b.get("bf3_work")
            if wk is None or wk.numel() < need:
                wk = b["bf3_work"] = torch.empty(need, dtype=torch.uint8, device=self.device)
        if sweep_events is not None:
            sweep_events[0].record()
        if l1q:  # TransE L1 count-only: the integer filter (same counts, bit for bit)
            e0, e1 = (0, self.n_ent) if entity_range is None else (int(entity_range[0]), int(entity_range[1]))
            call("mmre_link_sweep_l1q", int(s.pred_kind), float(s.margin), ptr(self.ent_km), ptr(self.ent_rows),
                 self.n_ent, self.e_pad, e0, e1, ptr(b["q_km"]), ptr(b["q_rows"]), ptr(b["q_true"]), ptr(qr),
                 ptr(qmode), n, b["q_pad"], s.dim, ptr(th), ptr(tt), ptr(b["counts"]), ptr(b["truth"]), ptr(wk),
                 int(wk.numel()), st)
        elif raw:  # the same filter over the raw DistMult rows (ent_km written only by an overflow fallback)
            e0, e1 = (0, self.n_ent) if entity_range is None else (int(entity_range[0]), int(entity_range[1]))
            call("mmre_link_sweep_bf3_rows", self.model_id, int(s.pred_kind), float(s.margin), ptr(ent_rows),
                 self.n_ent, self.e_pad, e0, e1, ptr(self.ent_km), ptr(b["q_km"]), ptr(b["q_rows"]),
                 ptr(b["q_true"]), ptr(qr), ptr(qmode), n, b["q_pad"], s.dim, ptr(b["counts"]), ptr(b["truth"]),
                 ptr(wk), int(wk.numel()), st)
        elif bf3:  # DistMult / ComplEx count-only: the split-bf16 MFMA filter (same counts, bit for bit)
            e0, e1 = (0, self.n_ent) if entity_range is None else (int(entity_range[0]), int(entity_range[1]))
            call("mmre_link_sweep_bf3", self.model_id, int(s.pred_kind), float(s.margin), ptr(self.ent_km),
                 ptr(self.ent_rows), self.n_ent, self.e_pad, e0, e1, ptr(b["q_km"]), ptr(b["q_rows"]),
                 ptr(b["q_true"]), ptr(qr), ptr(qmode), n, b["q_pad"], s.dim, ptr(b["counts"]), ptr(b["truth"]),
                 ptr(wk), int(wk.numel()), st)
        elif entity_range is not None:
            if return_scores:
                raise ValueError("entity_range sweeps keep no score rows")
            call("mmre_link_sweep_range", self.model_id, int(s.pred_kind), float(s.margin), ptr(self.ent_km),
                 self.n_ent, self.e_pad, int(entity_range[0]), int(entity_range[1]), ptr(b["q_km"]), ptr(b["q_true"]),
                 ptr(qr), ptr(qmode), n, b["q_pad"], s.dim, ptr(th), ptr(tt), ptr(b["counts"]), ptr(b["truth"]), st)
        else:
            call("mmre_link_sweep", self.model_id, int(s.pred_kind), float(s.margin), ptr(self.ent_km), self.n_ent,
                 self.e_pad, ptr(b["q_km"]), ptr(b["q_true"]), ptr(qr), ptr(qmode), n, b["q_pad"], s.dim, ptr(th),
                 ptr(tt), ptr(b["counts"]), ptr(b["truth"]), ptr(scores), st)
        if sweep_events is not None:
            sweep_events[1].record()
        b["l1q_used"] = l1q
        b["bf3_used"] = bf3
        b["bf3_raw"] = raw
        return dict(counts=b["counts"], truth=b["truth"], scores=scores)

    def _fusable(self, filt, type_masks, return_scores, prepare, sweep_events, q_rows):
        """The fused TransE L1 evaluation (mmre_link_evaluate_l1q) covers count-only runs with
        filter groups, no type masks, prediction = the score, the entity table prepared in the
        same call; sweep_events (the sweep kernel alone) keep the separate launches.
        MMRE_FUSED_EVAL=0 keeps the separate path (A/B)."""
        return (self.model_id == MODEL_IDS["transe"] and self.l1_filter and self.fused_eval and not return_scores
                and prepare and sweep_events is None and q_rows and type_masks is None and filt is not None
                and len(filt) == 5 and int(self.spec.pred_kind) == 0)

    def _run_fused(self, qh, qr, qt, qmode, filt, buffers, entity_range, undecided_q=None):
        s = self.spec
        n = int(qh.shape[0])
        b = buffers if buffers is not None else self.alloc_queries(n)
        gqo, gq, off, ids, entry_q = filt
        n_entries = int(ids.shape[0])
        lv = b.get("list_scores")
        if lv is None or lv.shape[0] < n_entries:
            lv = b["list_scores"] = torch.empty(max(n_entries, 1), dtype=torch.float32, device=self.device)
        need = int(_lib.lib().mmre_link_evaluate_l1q_workspace(s.dim, self.e_pad, b["q_pad"]))
        wk = b.get("l1q_work")
        if wk is None or wk.numel() < need or not b.get("l1q_work_zeroed"):
            # zeroed once: the call's grid tickets start at 0 and are left at 0
            wk = b["l1q_work"] = torch.zeros(need, dtype=torch.uint8, device=self.device)
            b["l1q_work_zeroed"] = True
        e0, e1 = (0, self.n_ent) if entity_range is None else (int(entity_range[0]), int(entity_range[1]))
        call("mmre_link_evaluate_l1q", int(bool(s.norm_flag)), ptr(self._ent), self.n_ent, ptr(self._rel), self.n_rel,
             s.dim, ptr(qh), ptr(qr), ptr(qt), ptr(qmode), n, ptr(gqo), ptr(gq), int(gqo.shape[0]) - 1, ptr(off),
             ptr(ids), ptr(entry_q), n_entries, e0, e1, ptr(self.ent_km), self.e_pad, ptr(self.ent_rows),
             ptr(b["q_km"]), b["q_pad"], ptr(b["q_rows"]), ptr(b["q_true"]), ptr(lv), ptr(b["counts"]),
             ptr(b["truth"]), ptr(undecided_q), ptr(wk), int(wk.numel()), stream_ptr(self.device))
        self.prepared = True
        b["l1q_used"] = True
        b["bf3_used"] = False
        return dict(counts=b["counts"], truth=b["truth"], scores=None)

    def bf3_stats(self, buffers):
        """The split-bf16 MFMA filter's record of the last run() on `buffers` (mmre_link_bf3_stats):
        dict(undecided=pairs rescored with the canonical chain, fallback=True if the pair list
        overflowed and the exact f32 sweep counted instead), or None if that run did not use the
        filter. Synchronises the stream."""
        if not buffers.get("bf3_used"):
            return None
        wk = buffers["bf3_work"]
        out = buffers.get("bf3_stats")
        if out is None:
            out = buffers["bf3_stats"] = torch.zeros(2, dtype=torch.int64, device=self.device)
        call("mmre_link_bf3_stats", ptr(wk), int(wk.numel()), ptr(out), stream_ptr(self.device))
        u, f = (int(x) for x in out.cpu())
        return dict(undecided=u, fallback=bool(f))

    def filter_stats(self, buffers):
        """Whichever count-only filter the last run() on `buffers` used: dict(kind="l1q" | "bf3",
        undecided=..., fallback=...), or None (the exact sweep ran)."""
        st = self.l1q_stats(buffers)
        if st is not None:
            return dict(kind="l1q", **st)
        st = self.bf3_stats(buffers)
        return None if st is None else dict(kind="bf3", **st)

    def l1q_stats(self, buffers):
        """The integer filter's record of the last run() on `buffers` (mmre_link_l1q_stats):
        dict(undecided=pairs rescored with the canonical chain, fallback=True if the sweep ran
        the f32 path because the codes were too coarse, bits=8 | 16 the code width the sweep
        used -- None on the fallback, guarded=list entries refused by the rescoring's range guard,
        always 0), or None if that run did not use the filter (not TransE
        L1, score-storing, MMRE_L1_FILTER=0). Synchronises the stream."""
        if not buffers.get("l1q_used"):
            return None
        wk = buffers["l1q_work"]
        out = buffers.get("l1q_stats")
        if out is None:
            out = buffers["l1q_stats"] = torch.zeros(4, dtype=torch.int64, device=self.device)
        call("mmre_link_l1q_stats", ptr(wk), int(wk.numel()), ptr(out), stream_ptr(self.device))
        u, w, g, o = (int(v) for v in out.cpu())
        # the code-width word: 0 = 8-bit codes, 1 = the f32 fallback, 2 = 16-bit codes; guarded =
        # undecided-list entries the rescoring refused as out of range (0 unless a defect)
        return dict(undecided=u, fallback=w == 1, bits={0: 8, 2: 16}.get(w), guarded=g, max_offset=o)


def _rows_view(c):
    """(4, n) int32 with unit element stride (row stride free): column slices of one
    (4, 2n) count table are passed to the C reduction without a copy."""
    c = np.asarray(c)
    if c.dtype != np.int32 or c.ndim != 2 or c.strides[1] != 4 or c.strides[0] % 4:
        c = np.ascontiguousarray(c, np.int32)
    return c


def link_metrics(head_counts: np.ndarray, tail_counts: np.ndarray):
    """Test.h:232-327 metric reduction (host C++ in libmmre, P14 float order).
    head_counts/tail_counts: (4, n) int32 = raw, filt, raw_tc, filt_tc."""
    h, t = _rows_view(head_counts), _rows_view(tail_counts)
    n = h.shape[1]
    if t.shape[1] != n or h.shape[0] != 4 or t.shape[0] != 4:
        raise ValueError("head/tail counts must both be (4, n)")
    stride = h.strides[0] // 4
    if t.strides[0] != h.strides[0]:
        h, t = np.ascontiguousarray(h), np.ascontiguousarray(t)
        stride = n
    out = np.zeros(20, np.float32)
    call("mmre_link_metrics", h.ctypes.data, t.ctypes.data, n, stride, out.ctypes.data)
    return {g: {m: float(out[5 * gi + mi]) for mi, m in enumerate(METRIC_NAMES)} for gi, g in enumerate(GROUPS)}


def evaluate_link_prediction(spec: ScoreSpec, test_h, test_r, test_t, index: FilterIndex | None = None,
                             type_constrain: bool = False):
    """Full OpenKE link-prediction evaluation in test order (testList sorted by (r, h, t),
    Reader.h:227). Returns (metrics dict, per-query counts (head, tail) as numpy)."""
    test_h, test_r, test_t = (np.asarray(x, np.int64) for x in (test_h, test_r, test_t))
    n = len(test_h)
    dev = spec.ent.device
    qh = np.concatenate([test_h, test_h])
    qr = np.concatenate([test_r, test_r])
    qt = np.concatenate([test_t, test_t])
    qm = np.concatenate([np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)])
    filt = None
    masks = None
    if index is not None:
        filt = tuple(torch.from_numpy(a).to(dev) for a in index.groups(qh, qr, qt, qm))
        if type_constrain:
            tm = index.type_masks()
            masks = tuple(torch.from_numpy(m).to(dev) for m in tm)
    sw = LinkSweep(spec)
    res = sw.run(*(torch.from_numpy(x).to(dev) for x in (qh, qr, qt)), torch.from_numpy(qm).to(dev), filt=filt,
                 type_masks=masks)
    counts = res["counts"].cpu().numpy()
    head, tail = counts[:, :n], counts[:, n:]
    return link_metrics(head, tail), (head, tail)
