"""Run the C2 production evaluation (bench.py's tables: 300 HIP trainer steps) N times with
nothing else in the process, for per-kernel A/B traces of the fused / separate paths:

    rocprofv3 --kernel-trace --stats -d <dir> -o run -- python scripts/trace_eval.py [N] [world W] [rank K]

With `world W rank K` the evaluation is rank K's share of the W-way relation-sharded C2
(cost-packed and in the sweep order bench.py uses: mmre.sharding.rank_order)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmre.link import HEAD, TAIL, FilterIndex, LinkSweep  # noqa: E402
from mmre.sharding import calibrate_weights, lpt_partition, rank_order  # noqa: E402
from mmre.workloads import train_transe, workload_spec, zs_workload  # noqa: E402

n_rep = int(sys.argv[1]) if len(sys.argv) > 1 else 50
world = int(sys.argv[3]) if len(sys.argv) > 3 else 1
rank = int(sys.argv[5]) if len(sys.argv) > 5 else 0
dev = torch.device("cuda:0")
w = zs_workload("FB15K-237-ZS", "transe", 200)
w["norm_flag"] = True
train_transe(w, dev, steps=300)
spec = workload_spec(w, dev)
index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
n = len(w["test_h"])
qh, qr, qt = (np.r_[w[k], w[k]] for k in ("test_h", "test_r", "test_t"))
qm = np.r_[np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)]
wts = calibrate_weights(spec, qh, qr, qt, qm, index, dev)   # the bench's packing and sweep order
m = rank_order(lpt_partition(qr, world, weights=wts)[rank], wts)
to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
q = [to(x[m]) for x in (qh, qr, qt, qm)]
filt = tuple(to(a) for a in index.groups(qh[m], qr[m], qt[m], qm[m]))
sw = LinkSweep(spec)
bufs = sw.alloc_queries(len(m))
torch.cuda.synchronize()
for _ in range(n_rep):
    sw.run(*q, filt=filt, buffers=bufs)
torch.cuda.synchronize()
print(f"{n_rep} evaluations of {len(m)} sweeps: {sw.filter_stats(bufs)}", flush=True)
