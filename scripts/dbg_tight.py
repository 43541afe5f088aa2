"""Debug: the tight L1 bound on the adversarial TransE table of test_sweep_filters_gpu (seed 0)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-relation-extrapolation_amd"), REPO, os.path.join(REPO, "tests"),
                os.path.join(REPO, "oracle")]
import numpy as np
import torch

os.environ["MMRE_L1_BITS"] = "8"
from test_sweep_filters_gpu import _adversarial
from test_link_gpu import _run, _spec_from
from mmre.link import FilterIndex

ent, rel, qh, qr, qt, qm = _adversarial(seed=0, margin=6.0, model="transe", huge=False)
E, R, d = ent.shape[0], rel.shape[0], rel.shape[1]
rng = np.random.default_rng(10)
fh, fr, ft = rng.integers(0, E, 3 * E), rng.integers(0, R, 3 * E), rng.integers(0, E, 3 * E)
fh, fr, ft = np.concatenate([fh, qh]), np.concatenate([fr, qr]), np.concatenate([ft, qt])
heads = [np.unique(np.concatenate([rng.choice(E, E // 3, replace=False), qh[qr == r]])) for r in range(R)]
tails = [np.unique(np.concatenate([rng.choice(E, E // 3, replace=False), qt[qr == r]])) for r in range(R)]
index = FilterIndex(fh, fr, ft, E, R, heads, tails)
spec = _spec_from("transe", ent, rel, margin=None, dim=d, norm=True)
exact = _run(spec, qh, qr, qt, qm, index=index, tc=True, scores=True)
for tight in ("1", "0", "1", "1"):
    os.environ["MMRE_L1_TIGHT"] = tight
    plain = _run(spec, qh, qr, qt, qm, index=index, tc=False, scores=False)
    d1 = plain["counts"][1].astype(np.int64) - exact["counts"][1]
    print(f"   filtered diff nonzero {np.count_nonzero(d1)}", flush=True)
    ex = (plain["counts"][1].astype(np.int64) - plain["counts"][0]) - (exact["counts"][1].astype(np.int64) - exact["counts"][0])
    sc = exact["scores"]
    th = exact["truth"]
    ties = (sc == th[:, None]).sum(1) - 1
    near = (np.abs(sc - th[:, None]) <= 1e-5 * np.abs(th[:, None])).sum(1) - 1
    nz = np.nonzero(ex)[0]
    print("   extra", ex[nz][:12].tolist(), "ties", ties[nz][:12].tolist(), "near", near[nz][:12].tolist(),
          "q%3", (nz % 3)[:12].tolist(), "mode", np.asarray(qm)[nz][:12].tolist(), flush=True)
    print("   corr exact", (exact["counts"][1].astype(np.int64) - exact["counts"][0])[nz][:12].tolist(), flush=True)
    for b in np.nonzero(d1)[0][:2]:
        print(f"   q {b}: plain raw/filt {plain['counts'][0][b]}/{plain['counts'][1][b]}, exact raw/filt "
              f"{exact['counts'][0][b]}/{exact['counts'][1][b]}, truth plain {plain['truth'][b]!r} exact {exact['truth'][b]!r}",
              flush=True)
    diff = plain["counts"][0].astype(np.int64) - exact["counts"][0]
    print(f"tight={tight}: raw diff nonzero {np.count_nonzero(diff)} of {len(diff)}, min {diff.min()} max {diff.max()}",
          flush=True)
    bad = np.nonzero(diff)[0][:5]
    for b in bad:
        s = exact["scores"][b]
        th = exact["truth"][b]
        print(f"  query {b}: truth {th!r}, exact count {exact['counts'][0][b]}, plain {plain['counts'][0][b]}, "
              f"#(s < th) {(s < th).sum()}, #(s == th) {(s == th).sum()}, nearest above {np.sort(s[s > th])[:3]}")
