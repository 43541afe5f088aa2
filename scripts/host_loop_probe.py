"""Where a small rank share's evaluation loop spends host time (diagnostic, not a measurement of
record): rank K's share of the W-way relation-sharded C2 evaluation (bench tables, cost-packed,
graph-replayed), timed as
  replay          host time for g.replay() to return (no sync)
  synced          replay + D2H + sync per evaluation
  pipe_nometrics  the bench's two-deep loop without the host metric reduction
  pipe            the bench's loop (metrics of i - 1 while i runs)
  metrics         the Test.h reduction alone on this host
usage: python scripts/host_loop_probe.py [world W rank K]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmre.link import HEAD, TAIL, FilterIndex, LinkSweep, link_metrics  # noqa: E402
from mmre.sharding import calibrate_weights, lpt_partition, rank_order  # noqa: E402
from mmre.workloads import train_transe, workload_spec, zs_workload  # noqa: E402

world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rank = int(sys.argv[4]) if len(sys.argv) > 4 else 3
dev = torch.device("cuda:0")
w = zs_workload("FB15K-237-ZS", "transe", 200)
w["norm_flag"] = True
train_transe(w, dev, steps=300)
spec = workload_spec(w, dev)
index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
n = len(w["test_h"])
qh, qr, qt = (np.r_[w[k], w[k]] for k in ("test_h", "test_r", "test_t"))
qm = np.r_[np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)]
wts = calibrate_weights(spec, qh, qr, qt, qm, index, dev)
m = rank_order(lpt_partition(qr, world, weights=wts)[rank], wts) if world > 1 else np.arange(2 * n)
to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
q = [to(x[m]) for x in (qh, qr, qt, qm)]
filt = tuple(to(a) for a in index.groups(qh[m], qr[m], qt[m], qm[m]))
sw = LinkSweep(spec)
bufs = sw.alloc_queries(len(m))
for _ in range(3):
    sw.run(*q, filt=filt, buffers=bufs)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    gc = sw.run(*q, filt=filt, buffers=bufs)["counts"]
torch.cuda.synchronize()
hosts = [torch.empty((4, len(m)), dtype=torch.int32, pin_memory=True) for _ in range(2)]
full = np.zeros((4, 2 * n), np.int32)
R = 200


def t_replay():
    torch.cuda.synchronize()
    ts = []
    for _ in range(R):
        t = time.perf_counter()
        g.replay()
        ts.append(time.perf_counter() - t)
        torch.cuda.synchronize()
    return np.median(ts) * 1e3


def t_synced():
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(R):
        g.replay()
        hosts[0].copy_(gc, non_blocking=True)
        torch.cuda.current_stream().synchronize()
    return (time.perf_counter() - t) / R * 1e3


def t_pipe(metrics: bool):
    torch.cuda.synchronize()
    done = [torch.cuda.Event(), torch.cuda.Event()]
    pend = None
    t = time.perf_counter()
    for i in range(R):
        g.replay()
        hosts[i & 1].copy_(gc, non_blocking=True)
        done[i & 1].record()
        if pend is not None:
            done[pend].synchronize()
            if metrics:
                link_metrics(full[:, :n], full[:, n:])
        pend = i & 1
    done[pend].synchronize()
    return (time.perf_counter() - t) / R * 1e3


def t_metrics():
    t = time.perf_counter()
    for _ in range(R):
        link_metrics(full[:, :n], full[:, n:])
    return (time.perf_counter() - t) / R * 1e3


for rep in range(2):
    print(f"world {world} rank {rank} ({len(m)} sweeps): replay {t_replay():.3f} ms (host) | synced {t_synced():.3f} | "
          f"pipe_nometrics {t_pipe(False):.3f} | pipe {t_pipe(True):.3f} | metrics {t_metrics():.3f} ms", flush=True)
