"""C2 A/B of the L1 filter's code widths on the bench's trained tables (zs_workload + train_transe
300 steps) and on the xavier-init tables: eager LinkSweep runs and the graph-replayed
ShardedLinkEvaluation, with each run's filter record (undecided pairs, code width) and time."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np
import torch

from mmre.link import FilterIndex, HEAD, TAIL, LinkSweep, ScoreSpec
from mmre.sharding import ShardedLinkEvaluation
from mmre.workloads import train_transe, zs_workload

dev = torch.device("cuda:0")


def run(w, tag):
    n = len(w["test_h"])
    to = lambda a, dt=np.int64: torch.from_numpy(np.asarray(a, dt)).to(dev)
    qh, qr, qt = (np.r_[w[k], w[k]] for k in ("test_h", "test_r", "test_t"))
    qm = np.r_[np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)]
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
    filt = tuple(to(a, a.dtype) for a in index.groups(qh, qr, qt, qm))
    spec = ScoreSpec(model="transe", ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=200, norm_flag=True, pred_kind=0)
    ref = None
    for bits in (None, "8", "16"):
        if bits is None:
            os.environ.pop("MMRE_L1_BITS", None)
        else:
            os.environ["MMRE_L1_BITS"] = bits
        sw = LinkSweep(spec)
        bufs = sw.alloc_queries(2 * n)
        ts = []
        for _ in range(12):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            sw.run(to(qh), to(qr), to(qt), to(qm, np.int8), filt=filt, buffers=bufs, sweep_events=ev)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        c = bufs["counts"].cpu().numpy().copy()
        ref = c if ref is None else ref
        print(f"{tag} bits={bits}: sweep {np.median(ts[2:]):.3f} ms {sw.l1q_stats(bufs)} counts equal {np.array_equal(c, ref)}",
              flush=True)
    os.environ.pop("MMRE_L1_BITS", None)
    ev = ShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev, graph=True)
    ev.run(); ev.run()
    print(f"{tag} graph-replayed evaluation: {ev.filter_stats()}", flush=True)


w = zs_workload("FB15K-237-ZS", "transe", 200)
w["norm_flag"] = True
run(w, "xavier")
train_transe(w, dev, steps=300)
run(w, "trained")
