#!/usr/bin/env python
"""A/B of the M3AE linear's tile modes (MMRE_M3AE_TILE = 128 | 64, read once per
process) on the encoder's shapes at the FB15K-237-ZS packed row count. Diagnostic only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO]
import torch  # noqa: E402

from mmre._lib import call, ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("M3AE_ROWS", "2261"))
st = stream_ptr(dev)
for name, k, n, epi in (("qkv", 384, 1152, 0), ("fc", 384, 384, 2), ("fc1", 384, 1536, 1), ("fc2", 1536, 384, 2)):
    a = torch.randn(M, k, device=dev)
    w = torch.randn(n, k, device=dev) / k ** 0.5
    b = torch.randn(n, device=dev)
    o = torch.randn(M, n, device=dev)
    f = lambda: call("mmre_m3ae_linear", epi, ptr(a), M, k, ptr(w), n, ptr(b), ptr(o), ptr(o), st)
    for _ in range(5):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{os.environ.get('MMRE_M3AE_TILE', 'auto'):5s} {name:4s} {M}x{k}->{n}: {us:7.2f} us  "
          f"{2.0 * M * k * n / us / 1e6:6.1f} TF")
