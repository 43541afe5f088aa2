"""Diagnostic: the L1 filter's undecided-pair record under eager and graph-replayed evaluations."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import torch  # noqa: E402

from mmre.link import FilterIndex  # noqa: E402
from mmre.sharding import ShardedLinkEvaluation  # noqa: E402
from mmre.workloads import train_transe, workload_spec, zs_workload  # noqa: E402

dev = torch.device("cuda:0")
w = zs_workload("FB15K-237-ZS", "transe", 200)
w["norm_flag"] = True
train_transe(w, dev, steps=300)
index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
spec = workload_spec(w, dev)
for graph in (False, True):
    ev = ShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev, graph=graph)
    for i in range(3):
        m, c = ev.run()
        wk = ev.sweep_buffers.get("l1q_work")
        raw = wk[256:256 + 16 * 256].view(torch.int64)[::32].cpu().tolist() if wk is not None else None
        print(f"graph={graph} run {i}: stats {ev.filter_stats()} slots {raw} hit10 {m['filter']['hit10']}", flush=True)

# the bench's sequence: two-deep pipelined evaluations, an eager twin sweep, then run + stats
ev = ShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev, graph=True)


def steps(k):
    pending = None
    for _ in range(k):
        t = ev.launch()
        if pending is not None:
            ev.finish(pending, copy_counts=False)
        pending = t
    if pending is not None:
        ev.finish(pending, copy_counts=False)


steps(10)
wk = ev.sweep_buffers["l1q_work"]
print("after warmup", [hex(x) for x in wk[256:256 + 16 * 256].view(torch.int64)[::32].cpu().tolist()], flush=True)
steps(100)
print("after 100", [hex(x) for x in wk[256:256 + 16 * 256].view(torch.int64)[::32].cpu().tolist()], flush=True)
from mmre.link import LinkSweep  # noqa: E402
sw = LinkSweep(spec)
bufs = sw.alloc_queries(len(ev.q_host[0]))
for _ in range(20):
    sw.run(*ev.q, filt=ev.filt, type_masks=ev.masks_tc, buffers=bufs)
torch.cuda.synchronize()
print("twin", sw.filter_stats(bufs), flush=True)
del sw, bufs
ev.run()
print("bench sequence:", ev.filter_stats(),
      [hex(x) for x in wk[256:256 + 16 * 256].view(torch.int64)[::32].cpu().tolist()], flush=True)
