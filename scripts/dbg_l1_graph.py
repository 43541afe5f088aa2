"""Debug: the L1 filter's header words (M, code width, probe count) across graph replays of the
bench's C2 evaluation, next to eager runs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np
import torch

from mmre.link import FilterIndex, LinkSweep, ScoreSpec
from mmre.sharding import ShardedLinkEvaluation
from mmre.workloads import train_transe, zs_workload

dev = torch.device("cuda:0")
w = zs_workload("FB15K-237-ZS", "transe", 200)
w["norm_flag"] = True
train_transe(w, dev, steps=300)
index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
spec = ScoreSpec(model="transe", ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=200, norm_flag=True, pred_kind=0)


def hdr(ev):
    wk = ev.sweep_buffers["l1q_work"]
    h = wk[:16].view(torch.int32).cpu().numpy()
    return f"M {np.frombuffer(h[:1].tobytes(), np.float32)[0]:.4f} width {h[1]} probe {h[2]}"


for graph in (False, True):
    ev = ShardedLinkEvaluation(spec, w["test_h"], w["test_r"], w["test_t"], index=index, device=dev, graph=graph)
    for i in range(4):
        m, c = ev.run()
        print(f"graph={graph} run {i}: {hdr(ev)} {ev.filter_stats()} hit10 {m['filter']['hit10']:.4f}", flush=True)
    tk = [ev.launch(), ev.launch()]
    ev.finish(tk[0]); ev.finish(tk[1])
    print(f"graph={graph} pipelined: {hdr(ev)} {ev.filter_stats()}", flush=True)
    pending = None
    for i in range(40):
        t = ev.launch()
        if pending is not None:
            ev.finish(pending)
        pending = t
    ev.finish(pending)
    print(f"graph={graph} after 40 pipelined: {hdr(ev)} {ev.filter_stats()}", flush=True)
    sw = LinkSweep(spec)
    bufs = sw.alloc_queries(len(ev.q_host[0]))
    for _ in range(3):
        sw.run(*ev.q, filt=ev.filt, type_masks=ev.masks_tc, buffers=bufs)
    torch.cuda.synchronize()
    print(f"graph={graph} eager twin: {sw.filter_stats(bufs)}", flush=True)
    del sw, bufs
    ev.run()
    print(f"graph={graph} after the twin: {hdr(ev)} {ev.filter_stats()}", flush=True)
