#!/usr/bin/env python
"""Diagnostic: time k_truth_filter alone on C2 under several groupings (events on the
launch stream). Not part of the measurement of record."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmre._lib import call, ptr, stream_ptr  # noqa: E402
from mmre.link import FilterIndex, LinkSweep, ScoreSpec  # noqa: E402
from mmre.workloads import zs_workload  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    w = zs_workload()
    index = FilterIndex(w["filter_h"], w["filter_r"], w["filter_t"], w["n_ent"], w["n_rel"])
    spec = ScoreSpec(model="transe", ent=w["ent"].to(dev), rel=w["rel"].to(dev), dim=200, norm_flag=True)
    n = len(w["test_h"])
    qh, qr, qt = (np.concatenate([w[k], w[k]]) for k in ("test_h", "test_r", "test_t"))
    qm = np.r_[np.zeros(n, np.int8), np.ones(n, np.int8)]
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    Q = [to(qh), to(qr), to(qt), to(qm)]
    sw = LinkSweep(spec)
    b = sw.alloc_queries(2 * n)
    sw.run(*Q, buffers=b)
    torch.cuda.synchronize()
    st = stream_ptr(dev)
    ident = tuple(to(a) for a in index.filters(qh, qr, qt, qm))

    def legacy(off, ids, qrow):
        call("mmre_link_truth", 0, 0, 0.0, ptr(sw.ent_km), sw.n_ent, sw.e_pad, ptr(sw.ent_rows), ptr(b["q_km"]),
             ptr(b["q_true"]), ptr(Q[1]), ptr(Q[3]), 2 * n, b["q_pad"], 200, ptr(off), ptr(ids), None, None,
             ptr(b["counts"]), ptr(b["truth"]), st)

    variants = {"per-query CSR, no lists": lambda: legacy(None, None, False),
                "per-query CSR, lists": lambda: legacy(*ident, False)}
    for mg in (1 << 30, 64, 16):
        g = [to(a) for a in index.groups(qh, qr, qt, qm, max_group=mg)]
        lv = torch.empty(g[3].shape[0], device=dev)

        def grouped(g=g, lv=lv):
            call("mmre_link_truth_grouped", 0, 0, 0.0, ptr(sw.ent_rows), sw.n_ent, ptr(b["q_rows"]),
                 ptr(b["q_true"]), ptr(Q[1]), ptr(Q[3]), 2 * n, 200, ptr(g[0]), ptr(g[1]), g[0].shape[0] - 1,
                 ptr(g[2]), ptr(g[3]), ptr(g[4]), g[3].shape[0], None, None, ptr(lv), ptr(b["counts"]),
                 ptr(b["truth"]), st)
        variants[f"groups max {mg} ({g[0].shape[0] - 1})"] = grouped
    for name, fn in variants.items():
        ts = []
        for it in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3)
        print(f"{name:32s}: {np.median(ts):8.1f} us")


if __name__ == "__main__":
    main()
