"""Relation-sharded multi-GPU evaluation.

Test relations are assigned to ranks by LPT packing of their query counts (a relation larger
than the per-rank share is first cut into contiguous query pieces), so every rank keeps
Test.h's relation-major order (testList sorted by (r, h, t), Reader.h:227) for its queries
and reuses its relations' rows. Entity and relation tables are replicated (11-60 MB at
the ZS configs, far below 288 GB). After the local sweep, ONE all-gather of the per-rank int32
rank-count lists (RCCL over xGMI; gloo on CPU in tests) lets every rank reduce the metrics in
the reference's sequential order, so rank 0's metrics are bit-equal to the single-GPU run.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def lpt_partition(rel_of_query: np.ndarray, world: int, split: bool = True, weights=None):
    """Assign the queries to `world` ranks by relation, heaviest relation first onto the
    least-loaded rank (LPT). With split (SURVEY.md §8(e)'s fallback) no rank takes more than
    the share ceil(Q / world): a relation that does not fit the least-loaded rank fills it with
    a contiguous run of its queries (query order) and the rest moves on -- at most world - 1
    cuts in all, and every rank's queries stay relation-major (Test.h's order). DB15K-ZS's
    largest relation holds 18 % of the queries, which caps whole-relation LPT at 5.4x on 8
    ranks. Deterministic (every rank computes the same partition). Returns one boolean mask
    over the queries per rank.

    weights (per query, > 0): pack by cost instead of by count (cost_weights: a query whose
    pairs the L1 filter leaves undecided costs more than its sweep), same rules with the
    share = total weight / world."""
    rel_of_query = np.asarray(rel_of_query)
    Q = len(rel_of_query)
    if Q == 0:
        return [np.zeros(0, bool) for _ in range(world)]
    if weights is not None:
        return _lpt_weighted(rel_of_query, world, split, np.asarray(weights, np.float64))
    share = -(-Q // world)
    order_q = np.argsort(rel_of_query, kind="stable")
    rels, starts, counts = np.unique(rel_of_query[order_q], return_index=True, return_counts=True)
    order = np.lexsort((rels, -counts))  # heaviest first, ties by relation id
    load = np.zeros(world, np.int64)
    own = np.zeros(Q, np.int64)
    for i in order:
        lo, left = int(starts[i]), int(counts[i])
        while left > 0:
            k = int(np.argmin(load))
            take = left if not split else min(left, max(share - int(load[k]), 0) or left)
            own[order_q[lo:lo + take]] = k
            load[k] += take
            lo += take
            left -= take
    return [own == k for k in range(world)]


def _lpt_weighted(rel_of_query, world, split, w):
    Q = len(rel_of_query)
    if w.shape != (Q,) or not np.all(w > 0):
        raise ValueError("lpt_partition: weights must be positive, one per query")
    share = float(w.sum()) / world
    order_q = np.argsort(rel_of_query, kind="stable")
    rels, starts, counts = np.unique(rel_of_query[order_q], return_index=True, return_counts=True)
    wq = w[order_q]
    cw = np.concatenate([[0.0], np.cumsum(wq)])                  # prefix weights in relation-major order
    rel_w = cw[starts + counts] - cw[starts]
    order = np.lexsort((rels, -rel_w))                            # heaviest first, ties by relation id
    load = np.zeros(world, np.float64)
    own = np.zeros(Q, np.int64)
    for i in order:
        lo, hi = int(starts[i]), int(starts[i] + counts[i])
        while lo < hi:
            k = int(np.argmin(load))
            room = share - load[k]
            rest = cw[hi] - cw[lo]
            if not split or rest <= room * (1 + 1e-9) or room <= 0:
                take = hi - lo
            else:  # the longest run of the relation's queries that fits the room (at least one)
                take = max(int(np.searchsorted(cw, cw[lo] + room, side="right")) - 1 - lo, 1)
            own[order_q[lo:lo + take]] = k
            load[k] += cw[lo + take] - cw[lo]
            lo += take
    return [own == k for k in range(world)]


def calibrate_weights(spec, qh, qr, qt, qm, index, device, group=None):
    """Per-query costs for the relation-sharded partition, from ONE evaluation of every query
    before any timing: the pairs the TransE L1 filter leaves undecided concentrate on some
    relations' queries (an 8-way share of C2 put 1.2 % of its pairs in the 8-bit band where the
    whole evaluation has 0.2 %), and each costs ~140 swept pairs. Rank 0's counts are broadcast
    so every rank packs the same partition. None (count-based packing) for other models."""
    import torch.distributed as dist
    from .link import LinkSweep
    if spec is None or index is None or spec.model != "transe":
        return None
    if len(qh) == 0:
        return None
    sw = LinkSweep(spec)
    if not sw._fusable((0,) * 5, None, False, True, None, True):
        return None
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    if not multi or dist.get_rank(group) == 0:  # the calibration runs on rank 0 only
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        filt = tuple(to(a) for a in index.groups(qh, qr, qt, qm))
        und = torch.zeros(len(qh), dtype=torch.int32, device=device)
        sw.run(to(qh), to(qr), to(qt), to(qm), filt=filt, undecided_q=und)
        w = torch.from_numpy(cost_weights(und.cpu().numpy(), sw.n_ent))
    else:
        w = torch.empty(len(qh), dtype=torch.float64)
    del sw
    if multi:  # every rank packs rank 0's costs
        t = w.to(device) if dist.get_backend(group) == "nccl" else w
        dist.broadcast(t, dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        w = t.cpu()
    return w.numpy()


# swept pairs one rescored pair costs (the L1 filter's canonical-chain rescoring of an undecided
# pair, ~200 dependent f32 operations on two gathered rows). 140 until the rescoring's count
# atomics were aggregated per query (round 6); 8-way C2 emulation, slowest rank: 140 0.198 ms,
# 90 0.187 ms (every rank 0.180-0.187), 60 0.251 ms (one rank's probe then picks 16-bit codes)
PAIR_COST = 90.0


def cost_weights(undecided_per_query, n_ent: int, pair_cost: float | None = None):
    """Per-query sweep cost for lpt_partition(weights=): the query's n_ent swept pairs plus
    pair_cost x its pairs the L1 filter left undecided (each gathered and rescored with the
    canonical chain: ~90 swept pairs' worth on MI355X, PAIR_COST), from one calibration
    evaluation (mmre_link_evaluate_l1q's per-query counters)."""
    if pair_cost is None:  # MMRE_PAIR_COST: A/B of the calibration constant
        pair_cost = float(os.environ.get("MMRE_PAIR_COST", PAIR_COST))
    u = np.asarray(undecided_per_query, np.float64)
    return float(n_ent) + pair_cost * u


def rank_order(mask, weights=None, tile: int = 128):
    """The query ids of one rank's share in sweep order. Without per-query costs: ascending
    (relation-major, Test.h order). With them (the calibration's undecided-pair counts): the
    heavy queries SPREAD over the sweep's query tiles -- ids sorted by cost, heaviest first, and
    dealt round-robin to the ceil(n / tile) tiles -- so every 128-query tile carries a like
    share of the pairs the L1 filter leaves undecided. The Test.h order puts a heavy relation's
    queries in the same few tiles, whose units then rescore for longest and trail the sweep;
    sorting heaviest-first made that worse (C2 8-way, slowest rank 0.277 -> 0.332 ms). Counts
    are per query, so the order changes no result. MMRE_RANK_ORDER=id|heavy|spread (A/B)."""
    ids = np.nonzero(mask)[0]
    mode = os.environ.get("MMRE_RANK_ORDER", "spread")
    if weights is None or mode == "id" or len(ids) == 0:
        return ids
    ids = ids[np.argsort(-np.asarray(weights, np.float64)[ids], kind="stable")]
    if mode == "heavy":
        return ids
    n_t = -(-len(ids) // tile)
    return np.concatenate([ids[t::n_t] for t in range(n_t)])


class ShardPlan:
    """Everything each rank precomputes once from the (deterministic, identical on every rank)
    lpt_partition masks: its own query ids (in rank_order), the padded width, and the device
    index maps that put all-gathered columns back into global query order."""

    def __init__(self, masks, device, weights=None):
        self.world = len(masks)
        self.n_total = len(masks[0])
        self.sizes = [int(m.sum()) for m in masks]
        self.pad = max(max(self.sizes), 1)
        self.ids = [rank_order(m, weights) for m in masks]
        # one gather from the all-gathered (world, 4, pad) block into (4, n_total) global order:
        # global column q of count row c <- flat index (rank(q) * 4 + c) * pad + local(q)
        src = np.empty((4, self.n_total), np.int64)
        for k in range(self.world):
            for c in range(4):
                src[c, self.ids[k]] = (k * 4 + c) * self.pad + np.arange(self.sizes[k])
        self.src = torch.from_numpy(src).to(device)
        self.bufs = {}    # persistent exchange buffers per evaluation slot (allocated on first use)
        self.device = device


def gather_counts(local_counts: torch.Tensor, plan: ShardPlan, group=None, slot: int = 0):
    """All-gather per-rank (4, n_local) int32 count lists into global query order: ONE
    collective of world x 4 x pad int32 (about 282 KB in total at FB15K-237-ZS), no index
    exchange (every rank knows the partition). `slot`: the evaluation slot whose exchange
    buffers to use (evaluations in flight on different streams must not share them)."""
    import torch.distributed as dist
    if slot not in plan.bufs:
        # persistent: the padding columns are never read (plan.src skips them), so no zeroing
        plan.bufs[slot] = (torch.empty((4, plan.pad), dtype=torch.int32, device=plan.device),
                           torch.empty((plan.world * 4, plan.pad), dtype=torch.int32, device=plan.device))
    buf, out = plan.bufs[slot]
    buf[:, :local_counts.shape[1]] = local_counts
    if buf.is_cuda and dist.get_backend(group) == "gloo":  # gloo (tests): the exchange goes through host memory
        host = torch.empty((plan.world * 4, plan.pad), dtype=torch.int32)
        dist.all_gather_into_tensor(host, buf.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, buf, group=group)  # rank-major concatenation along dim 0
    return torch.take(out, plan.src)   # (4, n_total) in global query order, one gather


class ShardedLinkEvaluation:
    """Relation-sharded filtered link prediction for one process of a torch.distributed job
    (one process per GPU; backend 'nccl' = RCCL over xGMI on MI355X, 'gloo' in CPU tests).

    Every rank builds the same LPT partition of the evaluation's queries (test triples x
    {head_batch, tail_batch}), sweeps only its own relations' queries, then one all-gather of
    the int32 rank counts gives every rank the full count table; the Test.h metric reduction
    then runs in the reference's sequential query order, so rank 0's metrics are bit-identical
    to a single-GPU evaluation. `local_runner(qh, qr, qt, qm, filt)` -> (4, n_local) int32
    device tensor is the per-rank sweep (defaults to mmre.link.LinkSweep).

    graph=True (default LinkSweep runner on a GPU): the rank's local evaluation -- entity and
    query prep, truth/filter kernels, sweep -- is captured once into a hipGraph and replayed,
    so its ~6 launches cost one; what a rank pays whatever its share shrinks.
    The all-gather and the D2H stay outside the graph. Timing events passed to counts() then
    bracket the whole replay, not the sweep kernel alone.

    streams=2 (default runner on a GPU): two evaluation slots, each with its own LinkSweep
    buffers, hipGraph, exchange buffers and HIP stream; launch() alternates them, so evaluation
    i + 1's short latency-bound kernels (prep, quantization, filter counts) run beside the tail
    of evaluation i's sweep instead of after it. Every evaluation still does all of its work
    from the raw tables; only independent evaluations overlap."""

    def __init__(self, spec, test_h, test_r, test_t, index=None, type_constrain=False, group=None,
                 device=None, local_runner=None, graph=False, cost=None, streams=1):
        import torch.distributed as dist
        from .link import HEAD, TAIL
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        th, tr, tt = (np.asarray(x, np.int64) for x in (test_h, test_r, test_t))
        self.n = len(th)
        qh, qr, qt = np.concatenate([th, th]), np.concatenate([tr, tr]), np.concatenate([tt, tt])
        qm = np.concatenate([np.full(self.n, HEAD, np.int8), np.full(self.n, TAIL, np.int8)])
        dev = torch.device(device) if device is not None else (spec.ent.device if spec is not None else
                                                               torch.device("cpu"))
        self.device = dev
        self.weights = None
        if cost == "undecided" and local_runner is None and not type_constrain:
            self.weights = calibrate_weights(spec, qh, qr, qt, qm, index, dev, group)
        self.masks = lpt_partition(qr, self.world, weights=self.weights)
        mine = rank_order(self.masks[self.rank], self.weights)   # this rank's query ids, sweep order
        self.order = mine
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self.q = [to(qh[mine]), to(qr[mine]), to(qt[mine]), to(qm[mine])]
        self.q_host = (qh[mine], qr[mine], qt[mine], qm[mine])
        self.filt = None
        self.masks_tc = None
        if index is not None:
            self.filt = tuple(to(a) for a in index.groups(qh[mine], qr[mine], qt[mine], qm[mine]))
            if type_constrain:
                tm = index.type_masks()
                if tm is None:
                    raise ValueError("type_constrain=True needs the FilterIndex's type constraints "
                                     "(type_constrain.txt, Reader.h:266-317)")
                self.masks_tc = tuple(to(m) for m in tm)
        self.plan = ShardPlan(self.masks, dev, self.weights) if self.world > 1 else None
        # one GPU with a cost order: the local columns go back to query order by one gather
        self._unperm = None
        if self.world == 1 and not np.array_equal(mine, np.arange(len(qh))):
            inv = np.empty(len(mine), np.int64)
            inv[mine] = np.arange(len(mine))
            self._unperm = to(inv)
        self._default_runner = local_runner is None
        n_slots = 2 if (streams > 1 and local_runner is None and dev.type == "cuda") else 1
        self._runners = [local_runner] * n_slots
        if local_runner is None:
            from .link import LinkSweep
            self._sweeps = []
            for j in range(n_slots):
                sw = LinkSweep(spec)
                bufs = sw.alloc_queries(len(mine))

                def run_slot(qh_, qr_, qt_, qm_, filt, masks_tc, events=None, sw=sw, bufs=bufs):
                    return sw.run(qh_, qr_, qt_, qm_, filt=filt, type_masks=masks_tc, buffers=bufs,
                                  sweep_events=events)["counts"]
                self._runners[j] = run_slot
                self._sweeps.append((sw, bufs))
            self.sweep, self.sweep_buffers = self._sweeps[0]
        self.local_runner = self._runners[0]
        self._streams = [torch.cuda.Stream(dev) for _ in range(n_slots)] if n_slots > 1 else None
        self._graph_wanted = bool(graph) and dev.type == "cuda" and self._default_runner
        self._graphs = [None] * n_slots
        self._graph_outs = [None] * n_slots

    def _local(self, events=None, slot=0):
        run = self._runners[slot]
        if not self._graph_wanted:
            return run(*self.q, self.filt, self.masks_tc, events)
        if self._graphs[slot] is None:
            # one eager run allocates every lazily sized buffer, then capture on a side stream
            run(*self.q, self.filt, self.masks_tc, None)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._graph_outs[slot] = run(*self.q, self.filt, self.masks_tc, None)
            self._graphs[slot] = g
        if events is not None:
            events[0].record()
        self._graphs[slot].replay()
        if events is not None:
            events[1].record()
        return self._graph_outs[slot]

    def counts(self, events=None):
        """(4, 2n) int32 counts in global query order (head block, then tail block), on the
        current stream (which first waits for slot 0's stream, whose buffers it reuses)."""
        if self._streams is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._streams[0])
        return self._counts(events, 0)

    def _counts(self, events=None, slot=0):
        self._last_slot = slot
        local = self._local(events, slot)
        if self.world > 1:
            return gather_counts(local, self.plan, self.group, slot)
        return local if self._unperm is None else local.index_select(1, self._unperm)

    def launch(self, events=None):
        """Enqueue one evaluation -- sweep, (world > 1) all-gather, and the D2H of the count
        table into a free one of two pinned buffers -- without waiting for it. Returns a ticket
        for finish(). Each ticket owns its buffer until it is finished (in any order), so at
        most two may be outstanding: the host metric reduction of evaluation i runs while the
        GPU sweeps i + 1."""
        free = getattr(self, "_free", None)
        if free is not None and not free:
            raise RuntimeError("ShardedLinkEvaluation: finish() a ticket before launching a third")
        if self._streams is not None:
            # the evaluation slot = the free pinned buffer; its stream first waits for whatever
            # the caller's stream has enqueued (the inputs)
            if free is None:
                self._free = free = [0, 1]
            slot = free[0]
            st = self._streams[slot]
            st.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(st):
                ticket = self._stage(self._counts(events, slot), st)
            return ticket
        c = self.counts(events)
        if not c.is_cuda:
            return [c.numpy(), None, None]
        return self._stage(c, torch.cuda.current_stream(c.device))

    def _stage(self, c, stream):
        """D2H of the count table into a free pinned buffer on `stream`; the ticket."""
        free = getattr(self, "_free", None)
        hosts = getattr(self, "_hosts", None)
        if hosts is None or hosts[0].shape != c.shape:
            if free is not None and len(free) != 2:
                raise RuntimeError("ShardedLinkEvaluation: count shape changed with tickets outstanding")
            hosts = self._hosts = [torch.empty(c.shape, dtype=c.dtype, pin_memory=True) for _ in range(2)]
            free = self._free = [0, 1]
        slot = free.pop(0)
        h = hosts[slot]
        h.copy_(c, non_blocking=True)
        done = torch.cuda.Event()
        done.record(stream)
        return [h, done, slot]

    def finish(self, ticket, copy_counts=True):
        """Wait for a launch() ticket's counts (its own event only) and run the Test.h metric
        reduction: (metrics, counts (4, 2n) int32). The ticket's pinned buffer is free again
        afterwards; copy_counts=False returns that buffer itself (valid until the next launch)."""
        from .link import link_metrics
        c, done, slot = ticket
        if c is None:
            raise RuntimeError("ShardedLinkEvaluation: this ticket was already finished")
        ticket[0] = None
        if done is not None:
            done.synchronize()
            c = c.numpy()
            if copy_counts:
                c = c.copy()
            self._free.append(slot)
        return link_metrics(c[:, :self.n], c[:, self.n:]), c

    def run(self, events=None, copy_counts=True):
        """(metrics, counts (4, 2n) int32) of one evaluation, synchronously."""
        return self.finish(self.launch(events), copy_counts)

    def _last_sweep(self):
        """(LinkSweep, buffers) of the slot that ran the last local evaluation, with the current
        stream ordered after that slot's stream (its workspace is then complete and not in
        flight when a stats kernel reads it), or (None, None)."""
        sweeps = getattr(self, "_sweeps", None)
        if not sweeps:
            return None, None
        slot = getattr(self, "_last_slot", 0)
        if self._streams is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._streams[slot])
        return sweeps[slot]

    def l1q_stats(self):
        """The TransE L1 integer filter's record of this rank's last local sweep (undecided pairs,
        fallback), or None (another model / runner)."""
        sw, bufs = self._last_sweep()
        return None if sw is None else sw.l1q_stats(bufs)

    def filter_stats(self):
        """The count-only filter's record of this rank's last local sweep (LinkSweep.filter_stats:
        kind l1q / bf3, undecided pairs, fallback), or None."""
        sw, bufs = self._last_sweep()
        return None if sw is None else sw.filter_stats(bufs)


def entity_slices(n_ent: int, world: int, tile: int = 128):
    """Contiguous entity slices [e0, e1) per rank, cut at multiples of the sweep's entity tile:
    rank k owns tiles [k T / W, (k + 1) T / W) of the T = ceil(E / tile) tiles."""
    n_t = -(-int(n_ent) // tile)
    out = []
    for k in range(world):
        t0, t1 = k * n_t // world, (k + 1) * n_t // world
        out.append((t0 * tile, min(t1 * tile, int(n_ent))))
    return out


def reduce_counts(counts: torch.Tensor, group=None):
    """Sum each rank's (4, Q) int32 counts over the group in place: ONE all-reduce (RCCL under
    'nccl'; through host memory under 'gloo'). Integer sums are exact, so the result is the
    whole-table count table bit for bit."""
    import torch.distributed as dist
    if counts.is_cuda and dist.get_backend(group) == "gloo":
        host = counts.cpu()
        dist.all_reduce(host, group=group)
        counts.copy_(host)
    else:
        dist.all_reduce(counts, group=group)
    return counts


class EntityShardedLinkEvaluation(ShardedLinkEvaluation):
    """Entity-sharded filtered link prediction (the alternative for huge E): every
    rank sweeps ALL queries against its contiguous 1/world of the entity tiles (the table itself
    stays replicated for the truth scores), with filter lists restricted to its slice, and one
    all-reduce (sum) of the int32 count table gives every rank the whole-table counts; the
    Test.h reduction then runs in the reference's order, bit-identical to one GPU. Same
    launch / finish / run API as ShardedLinkEvaluation. Per-rank work is E / world per query
    whatever the relation mix; the price is the truth pass and query prep of every query on
    every rank, and an all-reduce of 4 x Q int32 instead of an all-gather of each rank's share."""

    def __init__(self, spec, test_h, test_r, test_t, index=None, type_constrain=False, group=None, device=None):
        import torch.distributed as dist
        from .link import HEAD, TAIL, LinkSweep
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        th, tr, tt = (np.asarray(x, np.int64) for x in (test_h, test_r, test_t))
        self.n = len(th)
        qh, qr, qt = np.concatenate([th, th]), np.concatenate([tr, tr]), np.concatenate([tt, tt])
        qm = np.concatenate([np.full(self.n, HEAD, np.int8), np.full(self.n, TAIL, np.int8)])
        dev = torch.device(device) if device is not None else spec.ent.device
        self.device = dev
        n_ent = int(spec.ent.shape[0])
        self.slices = entity_slices(n_ent, self.world)
        self.entity_range = self.slices[self.rank]
        self.masks = [np.ones(2 * self.n, bool) for _ in range(self.world)]  # every rank: every query
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self.q = [to(qh), to(qr), to(qt), to(qm)]
        self.filt = None
        self.masks_tc = None
        if index is not None:
            self.filt = tuple(to(a) for a in index.groups(qh, qr, qt, qm, entity_range=self.entity_range))
            if type_constrain:
                tm = index.type_masks()
                if tm is None:
                    raise ValueError("type_constrain=True needs the FilterIndex's type constraints "
                                     "(type_constrain.txt, Reader.h:266-317)")
                self.masks_tc = tuple(to(m) for m in tm)
        self.plan = None
        self._default_runner = False
        self._graph_wanted = False
        self._streams = None
        sw = LinkSweep(spec)
        bufs = sw.alloc_queries(2 * self.n)
        e0, e1 = self.entity_range

        def local_runner(qh_, qr_, qt_, qm_, filt, masks_tc, events=None):
            if e1 <= e0:  # more ranks than entity tiles: this rank's slice is empty
                if events is not None:
                    events[0].record()
                    events[1].record()
                return torch.zeros((4, 2 * self.n), dtype=torch.int32, device=dev)
            return sw.run(qh_, qr_, qt_, qm_, filt=filt, type_masks=masks_tc, buffers=bufs, sweep_events=events,
                          entity_range=(e0, e1))["counts"]
        self.local_runner = local_runner

    def counts(self, events=None):
        local = self.local_runner(*self.q, self.filt, self.masks_tc, events)
        return reduce_counts(local, self.group) if self.world > 1 else local
