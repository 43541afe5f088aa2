"""A/B timing of the C2 sweep kernel in this process (events around mmre_link_sweep)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np
import torch

from mmre.link import FilterIndex, LinkSweep, ScoreSpec
from mmre.workloads import zs_workload

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
model, dim, ds, norm = {"c2": ("transe", 200, "FB15K-237-ZS", True), "c3": ("complex", 200, "DB15K-ZS", False),
                        "c4": ("rotate", 512, "FB15K-237-ZS", False),
                        "c5": ("distmult", 256, "synthetic-1M", False)}[cfg]
if cfg == "c5":
    from mmre.workloads import synthetic_large
    w = synthetic_large()
else:
    w = zs_workload(ds, model, dim)
dev = torch.device("cuda:0")
n = len(w["test_h"])
qh = np.r_[w["test_h"], w["test_h"]]; qr = np.r_[w["test_r"], w["test_r"]]; qt = np.r_[w["test_t"], w["test_t"]]
qm = np.r_[np.zeros(n, np.int8), np.ones(n, np.int8)]
to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
from mmre.link import rotate_phase_denom
spec = ScoreSpec(model=model, ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=dim,
                 ent_im=w["ent_im"].to(dev) if "ent_im" in w else None,
                 rel_im=w["rel_im"].to(dev) if "rel_im" in w else None, norm_flag=norm,
                 pred_kind={"transe": 0, "complex": 2, "rotate": 3, "distmult": 2}[model], margin=float(w.get("margin", 0)),
                 phase_denom=rotate_phase_denom(6.0, 2.0, dim) if model == "rotate" else 0.0)
sw = LinkSweep(spec)
b = sw.alloc_queries(2 * n)
args = [to(qh), to(qr), to(qt), to(qm)]
ts = []
for i in range(reps + 3):
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    sw.run(*args, buffers=b, sweep_events=ev)
    torch.cuda.synchronize()
    if i >= 3:
        ts.append(ev[0].elapsed_time(ev[1]))
c = b["counts"].cpu().numpy()
print(f"{os.environ.get('TAG', '')} {cfg} sweep ms median {np.median(ts):.3f} min {np.min(ts):.3f} "
      f"checksum {int(c[0].sum())}")
