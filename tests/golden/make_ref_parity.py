"""make_ref_parity.py -- full-size, non-degenerate reference-rank fixtures for C3 / C4 / C5.

Runs only in the build container (it needs oracle/_ref/Base.so, compiled from
/root/reference/OpenKE/openke/base/Base.cpp by oracle/Makefile). Nothing from the reference
travels: only the numbers written to tests/golden/ref_parity_<config>.npz.

For each config the workload is mmre.workloads.ref_parity_workload(config): the bench's
workload (real DB15K-ZS / FB15K-237-ZS test triples, or C5's synthetic 1 M entities) with
STRUCTURED tables (mmre.workloads.structured_tables: deterministic, bit-identical on every
host, truths ranked near the top -- hit@10 ~0.5-0.8, not the ~0 of OpenKE-initialised tables)
and a seeded test sample:

    C2  FB15K-237-ZS TransE d=200   all 17,596 test triples -> 35,192 sweeps x 14,208 entities
        (norm_flag; the bench's TRAINED tables: 300 steps of this build's HIP trainer, written by
        scripts/dump_trained_tables.py on a GPU box, sha256 checked here and in the GPU test)
    C3  DB15K-ZS ComplEx d=200      all 5,653 test triples  -> 11,306 sweeps x 12,741 entities
    C4  FB15K-237-ZS RotatE d=512   all 17,596 test triples -> 35,192 sweeps x 14,208 entities
    C5  synthetic DistMult d=256    all 4,096 test triples  ->  8,192 sweeps x 1,000,000 entities

The REFERENCE's CPU path ranks the sample: the OpenKE Tester loop (Tester.py:70-91) over the
reference's own Base.so (the sample cut into contiguous chunks, one child process each:
ref_tester.run_parallel) (getHeadBatch / testHead / getTailBatch / testTail /
test_link_prediction, Test.h:36-327) with the reference models' predict op sequences on torch
CPU (oracle/ref_tester.py, pinned bit-for-bit against the reference's own predictions by
tests/test_oracle_golden.py). Stored per fixture:

    tables_sha256          identity of the structured tables (the GPU test rebuilds and checks them)
    sample, q              sample indices into the workload's Test.h-ordered test list; (h, r, t)
    counts (2, n, 2)       Base.so's per-query [raw, filtered] counts (rank - 1), [head | tail]
    truth_scores (2, n)    the reference's predict value of the truth
    score_absmax (2, n)    max |predict| over the sweep
    near_off/ids/scores    per sweep (head sweeps then tail sweeps), every other entity whose
                           reference score lies within near_rel x max|predict| of the truth's
    metrics                filtered MRR, MR, hit@10, hit@3, hit@1 of the whole sample: the Test.h
                           reduction of the merged counts (oracle.link_metrics), which reproduces
                           every chunk's Base.so getTestLink* bit for bit (chunk_metrics, chunk_n)

tests/test_ref_parity_gpu.py holds the HIP sweep to these exactly (see there).

Usage:  python tests/golden/make_ref_parity.py [c2 c3 c4 c5]   (C4: 1.4-3.9 s per test triple per
        process: 9,918 s for all 17,596 on 7 processes of an 8-CPU container; MMRE_REF_PROCS sets
        the process count)
        (c2 reads gpurun_out/trained_c2.npz)
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(REPO, "multimodal-relation-extrapolation_amd"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)

NEAR_REL = 1e-5


def make(config: str, procs: int = 8, tables_path: str | None = None):
    import ref_tester
    from mmre.workloads import TRAINED_TABLES, ref_parity_workload, tables_sha256
    t0 = time.time()
    if config in TRAINED_TABLES and tables_path is None:
        tables_path = os.path.join(REPO, "gpurun_out", f"trained_{config}.npz")
    w = ref_parity_workload(config, tables_path=tables_path)
    sha = tables_sha256(w)
    if tables_path is not None:
        with np.load(tables_path, allow_pickle=False) as z:
            assert str(z["sha256"]) == sha, "trained tables' sha256 differs from the one the GPU run recorded"
    print(f"{config}: workload + structured tables in {time.time() - t0:.1f} s, sha256 {sha[:16]}", flush=True)
    res = ref_tester.run_parallel(w, w["test_h"], w["test_r"], w["test_t"], procs, summary=True, near_rel=NEAR_REL)
    print(f"{config}: {len(res['q'])} test triples on {procs} processes, slowest chunk {float(res['elapsed']):.1f} s",
          flush=True)
    q = res["q"]
    assert np.array_equal(q[:, 0], w["test_h"]) and np.array_equal(q[:, 1], w["test_r"]) \
        and np.array_equal(q[:, 2], w["test_t"]), "Base.so's testList order differs from the workload's"
    out = dict(config=np.array(config), tables_sha256=np.array(sha), sample=w["sample"].astype(np.int32),
               q=q.astype(np.int32), counts=res["counts"].astype(np.int32),
               truth_scores=res["truth_scores"], score_absmax=res["score_absmax"],
               near_rel=np.float64(NEAR_REL), near_off=res["near_off"], near_ids=res["near_ids"],
               near_scores=res["near_scores"], metrics=res["metrics"], chunk_metrics=res["chunk_metrics"],
               chunk_n=res["chunk_n"], ref_elapsed_s=res["elapsed"], ref_threads=res["threads"], n_ent=res["n_ent"])
    path = os.path.join(HERE, f"ref_parity_{config}.npz")
    np.savez_compressed(path, **out)
    c = res["counts"][:, :, 1]
    print(f"{config}: {2 * len(q)} sweeps, filtered hit@1/3/10 {np.mean(c < 1):.3f} / {np.mean(c < 3):.3f} / "
          f"{np.mean(c < 10):.3f}, metrics {res['metrics'].tolist()}, near-tie sweeps "
          f"{int((np.diff(res['near_off']) > 0).sum())}, {os.path.getsize(path) / 1e3:.0f} kB", flush=True)


if __name__ == "__main__":
    for cfg in (sys.argv[1:] or ["c3", "c4", "c5"]):
        make(cfg, procs=int(os.environ.get("MMRE_REF_PROCS", "8")))
