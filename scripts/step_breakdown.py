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
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
