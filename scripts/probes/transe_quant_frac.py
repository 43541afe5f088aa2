"""Diagnostic: how many (query, entity) pairs of the C2 evaluation would a 16-bit integer
L1 filter (v_sad_u16 over quantized planes) leave undecided?

Builds the bench's C2 workload (FB15K-237-ZS TransE d 200, tables trained 300 steps by this
build's trainer), scores a sample of sweeps exactly (float64), and counts the pairs whose
score lies within the filter's worst-case error bound of the truth's score:
    B = K * delta (+ 2^-22 K S for the f32 chains), delta = 2 M / 65535, M = max |x|.
Prints the undecided fraction per pair and the probability that a wave's 4,096 pairs of a
unit hold at least one (each such wave rescores exactly). Needs a GPU (trainer)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "multimodal-relation-extrapolation_amd"))

from mmre.workloads import train_transe, zs_workload  # noqa: E402


def main():
    w = zs_workload("FB15K-237-ZS", "transe", 200)
    w["norm_flag"] = True
    train_transe(w, "cuda:0", steps=300)
    ent = w["ent"].double()
    rel = w["rel"].double()
    ent = ent / ent.norm(dim=1, keepdim=True).clamp_min(1e-12)
    rel = rel / rel.norm(dim=1, keepdim=True).clamp_min(1e-12)
    h, r, t = (np.asarray(w[k]) for k in ("test_h", "test_r", "test_t"))
    rng = np.random.default_rng(0)
    idx = rng.choice(len(h), 300, replace=False)
    K = 200
    qs, ths = [], []
    for i in idx:
        qs.append(ent[h[i]] + rel[r[i]]); ths.append(int(t[i]))    # tail batch
        qs.append(ent[t[i]] - rel[r[i]]); ths.append(int(h[i]))    # head batch
    Q = torch.stack(qs)
    M = max(float(Q.abs().max()), float(ent.abs().max()))
    S = torch.cdist(Q, ent, p=1)                                    # (2n, E)
    th = S[torch.arange(len(ths)), torch.tensor(ths)]
    for name, m, levels in (("16-bit, M = data max", M, 65535), ("16-bit, M = 2 (fixed bound)", 2.0, 65535),
                            ("8-bit, M = data max", M, 255), ("10-bit, M = data max", M, 1023)):
        delta = 2 * m / levels
        B = K * delta + 2.0 ** -22 * K * th
        und = ((S - th[:, None]).abs() <= B[:, None]).double()
        p = float(und.mean())
        print(f"{name}: M {m:.4f} delta {delta:.3g} bound/score {float((B / th).mean()):.3g}  undecided "
              f"fraction {p:.3g}  P(wave of 4096 pairs has one) {1 - (1 - p) ** 4096:.3f}  "
              f"mean rank of truth {float((S < th[:, None]).double().sum(1).mean()):.1f}")


if __name__ == "__main__":
    main()
