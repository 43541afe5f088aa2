#!/usr/bin/env python
"""Where the bench step's time goes (C2 by default): full step vs GPU launches + sync vs
D2H + host metric reduction. Diagnostic only; bench.py is the measurement of record."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmre.link import FilterIndex, ScoreSpec, link_metrics  # noqa: E402
from mmre.sharding import ShardedLinkEvaluation  # noqa: E402
from mmre.workloads import zs_workload  # noqa: E402


def timeit(fn, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="time one rank's share of a W-way relation-sharded step (no collective)")
    ap.add_argument("--entity", action="store_true", help="--emulate-world: entity-sharded ranks (all queries "
                    "against 1/W of the entity tiles) instead of query-sharded")
    ap.add_argument("--graph", action="store_true", help="--emulate-world: replay each rank's local evaluation "
                    "from a hipGraph")
    ap.add_argument("--pack", default="cost", choices=["cost", "count"],
                    help="--emulate-world: LPT by calibrated per-query cost (bench default) or by query count")
    ap.add_argument("--streams", type=int, default=2, choices=[1, 2],
                    help="--emulate-world --graph: evaluation slots on separate streams (bench.py --eval-streams)")
    ap.add_argument("--no-order", action="store_true",
                    help="--emulate-world: keep each rank's queries ascending (default: heaviest calibrated cost first)")
    ap.add_argument("--ranks", default="",
                    help="--emulate-world: comma-separated ranks to measure (default: all; N = 1 always runs)")
    ap.add_argument("--no-n1", action="store_true", help="--emulate-world: skip the N = 1 reference run")
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="--emulate-world: workload (c2: the bench's trained TransE tables; c3-c5: the "
                         "structured tables of the reference fixtures)")
    a = ap.parse_args()
    if a.emulate_world:
        return emulate(a)
    dev = torch.device("cuda:0")
    w = zs_workload()
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
    spec = ScoreSpec(model="transe", ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=200, norm_flag=True)
    ev = ShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev)
    for _ in range(3):
        ev.run(copy_counts=False)
    full = timeit(lambda: ev.run(copy_counts=False), a.reps)
    gpu = timeit(lambda: ev.counts(), a.reps)
    host = torch.empty((4, 2 * ev.n), dtype=torch.int32, pin_memory=True)

    def with_copy():
        host.copy_(ev.counts(), non_blocking=True)
        torch.cuda.current_stream().synchronize()
    d2h = timeit(with_copy, a.reps)
    empty = timeit(lambda: torch.cuda.current_stream().synchronize(), a.reps)
    c = ev.counts().cpu().numpy()
    n = ev.n
    t = time.perf_counter()
    for _ in range(a.reps):
        link_metrics(c[:, :n], c[:, n:])
    met = (time.perf_counter() - t) / a.reps * 1e3
    # host-side launch cost of one evaluation (no sync), and the metric reduction on pinned views
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        ev.counts()
    launch = (time.perf_counter() - t) / a.reps * 1e3
    torch.cuda.synchronize()
    hv = host.numpy()
    t = time.perf_counter()
    for _ in range(a.reps):
        link_metrics(hv[:, :n], hv[:, n:])
    met_pinned = (time.perf_counter() - t) / a.reps * 1e3
    print(f"launch-only (host) {launch:.3f} ms | metrics on pinned views {met_pinned:.3f} ms")
    print(f"full step {full:.3f} ms | launches+GPU {gpu:.3f} ms | +D2H+sync {d2h:.3f} ms | "
          f"host metrics {met:.3f} ms | empty sync {empty:.4f} ms")


# The RCCL all-gather of the count lists (world x 4 x pad int32, ~0.56 MB in all at C2) over
# xGMI at 8 ranks, which a one-GPU box cannot run: a latency-bound ring of 7 steps of ~70 KB; an
# estimate, stated as one wherever it is used.
EST_ALLGATHER_MS = 0.030


def emulate(a):
    """Per-rank cost of a W-way relation-sharded C2 step on this one GPU: each rank's LPT share
    swept and reduced alone (the all-gather is not included)."""
    from mmre.link import HEAD, TAIL, LinkSweep
    from mmre.sharding import lpt_partition
    from mmre.workloads import REF_PARITY, structured_tables, synthetic_large, train_transe, workload_spec
    dev = torch.device("cuda:0")
    (dataset, model, dim), _, _ = REF_PARITY[a.config]
    w = synthetic_large(dim=dim) if dataset == "synthetic-1M" else zs_workload(dataset, model, dim)
    if a.config == "c2":
        w["norm_flag"] = True
        train_transe(w, dev, steps=300)  # the bench's tables
    else:
        structured_tables(w)
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
    spec = workload_spec(w, dev)
    th, tr, tt = (np.asarray(x, np.int64) for x in (w["test_h"], w["test_r"], w["test_t"]))
    n = len(th)
    qh, qr, qt = np.concatenate([th, th]), np.concatenate([tr, tr]), np.concatenate([tt, tt])
    qm = np.concatenate([np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)])
    from mmre.sharding import entity_slices
    weights = None
    if a.pack == "cost" and not a.entity:  # the bench's packing: one calibration evaluation's per-query costs
        from mmre.sharding import calibrate_weights
        weights = calibrate_weights(spec, qh, qr, qt, qm, index, dev)
    masks = lpt_partition(qr, a.emulate_world, weights=weights)
    print(f"packing: {'cost-weighted (calibrated undecided pairs)' if weights is not None else 'query count'}")
    slices = entity_slices(w["n_ent"], a.emulate_world)
    if a.entity:
        masks = [np.ones(2 * n, bool)] * a.emulate_world
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    worst = worst_x = 0.0
    if a.emulate_world > 1:  # N = 1 under the same harness, for the ratio
        masks = [np.ones(2 * n, bool)] + list(masks)
        slices = [(0, w["n_ent"])] + list(slices)
    one = None
    from mmre.sharding import rank_order
    only = {int(x) for x in a.ranks.split(",") if x.strip()} if a.ranks else None
    for k, m in enumerate(masks):
        er = slices[k] if a.entity else None
        r_id = k - (1 if a.emulate_world > 1 else 0)
        if a.emulate_world > 1 and ((k == 0 and a.no_n1) or (k > 0 and only is not None and r_id not in only)):
            continue
        m = rank_order(m, None if a.no_order else weights)  # the rank's queries in the bench's sweep order
        q = [to(x[m]) for x in (qh, qr, qt, qm)]
        filt = tuple(to(x) for x in index.groups(qh[m], qr[m], qt[m], qm[m], entity_range=er))
        sw = LinkSweep(spec)
        bufs = sw.alloc_queries(len(m))
        host = torch.empty((4, len(m)), dtype=torch.int32, pin_memory=True)
        ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]

        def step():
            # the production call (fused TransE L1 evaluation where it applies: no sweep events)
            c = sw.run(*q, filt=filt, buffers=bufs, entity_range=er)["counts"]
            host.copy_(c, non_blocking=True)
            torch.cuda.current_stream().synchronize()
        for _ in range(3):
            step()
        if a.graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                gc = sw.run(*q, filt=filt, buffers=bufs, entity_range=er)["counts"]

            def step():
                g.replay()
                host.copy_(gc, non_blocking=True)
                torch.cuda.current_stream().synchronize()
            for _ in range(3):
                step()
        ms_sync = timeit(step, a.reps)
        # the bench's loop (bench.py steps(), ShardedLinkEvaluation.launch / finish): evaluation
        # i is enqueued (graph replay + D2H of its counts into one of two pinned buffers), then
        # the host waits for evaluation i - 1 and runs the Test.h metric reduction of the WHOLE
        # count table (every rank reduces the gathered 4 x 2n table; here a full-size stand-in),
        # so evaluation i runs while the host reduces i - 1. With two streams (streams=2) the
        # evaluations alternate between two buffer sets / graphs / streams.
        # pinned, like the bench's (ShardedLinkEvaluation._stage): empty_like(host) is pageable memory,
        # whose D2H copy blocks the host and serialised the loop (0.357 vs 0.257 ms for the 8-way rank 3)
        hosts = [torch.empty(host.shape, dtype=host.dtype, pin_memory=True) for _ in range(2)]
        full = np.zeros((4, 2 * n), np.int32)
        slots = [(sw, bufs, g if a.graph else None, gc if a.graph else None)]
        if a.graph and a.streams == 2:
            sw_b = LinkSweep(spec)
            bufs_b = sw_b.alloc_queries(len(m))
            sw_b.run(*q, filt=filt, buffers=bufs_b, entity_range=er)
            torch.cuda.synchronize()
            g_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_b):
                gc_b = sw_b.run(*q, filt=filt, buffers=bufs_b, entity_range=er)["counts"]
            slots.append((sw_b, bufs_b, g_b, gc_b))
        ss = [torch.cuda.Stream() for _ in slots] if len(slots) > 1 else [torch.cuda.current_stream()]

        def looped(reps, n_slots):
            torch.cuda.synchronize()
            done = [torch.cuda.Event(), torch.cuda.Event()]
            t = time.perf_counter()
            pend = None
            for i in range(reps):
                j = i % n_slots
                s_w, b_w, g_w, c_w = slots[j]
                with torch.cuda.stream(ss[j]):
                    if g_w is not None:
                        g_w.replay()
                        c = c_w
                    else:
                        c = s_w.run(*q, filt=filt, buffers=b_w, entity_range=er)["counts"]
                    hosts[i & 1].copy_(c, non_blocking=True)
                    done[i & 1].record(ss[j])
                if pend is not None:
                    done[pend].synchronize()
                    link_metrics(full[:, :n], full[:, n:])
                pend = i & 1
            done[pend].synchronize()
            link_metrics(full[:, :n], full[:, n:])
            torch.cuda.synchronize()
            return (time.perf_counter() - t) / reps * 1e3
        looped(3, 1)
        ms1 = looped(max(a.reps, 50), 1)
        ms = ms1
        if len(slots) > 1:
            looped(3, 2)
            ms = looped(max(a.reps, 50), 2)
            assert np.array_equal(slots[0][3].cpu().numpy(), slots[1][3].cpu().numpy())
        # the count exchange's own kernels (copy into the all-gather buffer + the one gather into
        # global order; mmre.sharding.gather_counts) on this GPU; the RCCL all-gather itself cannot
        # run on one GPU: EST_ALLGATHER_MS stands in for it (see the summary line)
        xch = 0.0
        if a.emulate_world > 1 and not a.entity and k > 0:
            from mmre.sharding import ShardPlan
            plan = ShardPlan(list(masks[1:]), dev, None if a.no_order else weights)
            buf = torch.empty((4, plan.pad), dtype=torch.int32, device=dev)
            out = torch.zeros((plan.world * 4, plan.pad), dtype=torch.int32, device=dev)
            local = bufs["counts"]

            def exchange():
                buf[:, :local.shape[1]] = local
                return torch.take(out, plan.src)
            exchange()
            xch = timeit(exchange, 50)
        # the sweep kernel alone: events on the launch stream around it, eager twins of the
        # evaluation (the separate launches; the sweep kernel is the same one)
        # the same eager run also bracketed whole (events before and after the call), so the
        # rank's fixed cost = eager local evaluation - its sweep, both from the one run (>= 0)
        sw2 = LinkSweep(spec)
        b2 = sw2.alloc_queries(len(m))
        ts, fx, loc = [], [], []
        outer = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
        for _ in range(7):
            outer[0].record()
            sw2.run(*q, filt=filt, buffers=b2, sweep_events=ev, entity_range=er)
            outer[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
            loc.append(outer[0].elapsed_time(outer[1]))
            fx.append(loc[-1] - ts[-1])
        sweep = float(np.median(ts))
        fixed = float(np.median(fx))
        local_eager = float(np.median(loc))
        if a.emulate_world > 1 and k == 0:
            one = ms
            print(f"N=1: {len(m)} sweeps, local evaluation {ms:.3f} ms pipelined{' on 2 streams' if ms != ms1 else ''} "
                  f"(one stream {ms1:.3f}; {ms_sync:.3f} ms with a sync per evaluation)")
            continue
        worst = max(worst, ms)
        worst_x = max(worst_x, xch)
        fst = sw.filter_stats(bufs)
        print(f"rank {r_id if a.emulate_world > 1 else k}: {len(m)} sweeps, local evaluation {ms:.3f} ms pipelined "
              f"(one stream {ms1:.3f}) "
              f"({ms_sync:.3f} synced), eager local {local_eager:.3f} ms = sweep kernel {sweep:.3f} ms + fixed "
              f"{fixed:.3f} ms (same runs), exchange kernels "
              f"{xch:.3f} ms, filter {fst}")
    if one is not None and worst > 0:
        est = 0.0 if a.entity else EST_ALLGATHER_MS
        tot = worst + worst_x + est
        print(f"{a.config} world {a.emulate_world}{' entity-sharded' if a.entity else ''}{' (graph)' if a.graph else ''}: "
              f"slowest rank {worst:.3f} ms + exchange kernels {worst_x:.3f} ms + RCCL all-gather estimate "
              f"{est:.3f} ms = {tot:.3f} ms per evaluation; N=1 {one:.3f} ms: {one / worst:.2f}x before the "
              f"exchange, {one / tot:.2f}x with it (the host metric reduction overlaps the next evaluation, "
              f"as at N=1)")


if __name__ == "__main__":
    main()
