#!/usr/bin/env python
"""How the C2 L1 filter's undecided pairs spread over queries (the bench's trained tables): the
per-query rescored-pair counts of one fused evaluation (mmre_link_evaluate_l1q's und_q) --
concentrated queries make their count-column atomics a same-address serial chain."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmre.link import HEAD, TAIL, FilterIndex, LinkSweep  # noqa: E402
from mmre.workloads import train_transe, workload_spec, zs_workload  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    w = zs_workload("FB15K-237-ZS", "transe", 200)
    w["norm_flag"] = True
    train_transe(w, dev, steps=300)
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
    spec = workload_spec(w, dev)
    th, tr, tt = (np.asarray(w[k], np.int64) for k in ("test_h", "test_r", "test_t"))
    n = len(th)
    qh, qr, qt = np.r_[th, th], np.r_[tr, tr], np.r_[tt, tt]
    qm = np.r_[np.full(n, HEAD, np.int8), np.full(n, TAIL, np.int8)]
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    filt = tuple(to(a) for a in index.groups(qh, qr, qt, qm))
    und = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    sw = LinkSweep(spec)
    res = sw.run(to(qh), to(qr), to(qt), to(qm), filt=filt, undecided_q=und)
    u = und.cpu().numpy().astype(np.int64)
    c = res["counts"].cpu().numpy()
    s = np.sort(u)[::-1]
    print(f"queries {len(u)}, undecided pairs {u.sum()}, queries with any {int((u > 0).sum())}")
    print("top 20:", s[:20].tolist())
    for f in (0.5, 0.9, 0.99):
        k = int(np.searchsorted(np.cumsum(s), f * s.sum())) + 1
        print(f"{int(f * 100)} % of the pairs in the top {k} queries")
    print("raw count of the top-5 queries:", c[0][np.argsort(u)[::-1][:5]].tolist())


if __name__ == "__main__":
    main()
