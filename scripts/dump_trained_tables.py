"""dump_trained_tables.py -- (GPU) train the C2 tables the way bench.py does (300 steps of the
HIP trainer, mmre.workloads.train_transe) TWICE in one process, check the two results are
bit-identical, and write them to gpurun_out/trained_c2.npz with their sha256, so that
tests/golden/make_ref_parity.py can rank them with the reference's CPU path in the build
container (which has no GPU).

    python scripts/dump_trained_tables.py [out.npz]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multimodal-relation-extrapolation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmre.workloads import ref_parity_workload, tables_sha256  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "trained_c2.npz")
os.makedirs(os.path.dirname(out), exist_ok=True)
a = ref_parity_workload("c2", device="cuda:0")
b = ref_parity_workload("c2", device="cuda:0")
sa, sb = tables_sha256(a), tables_sha256(b)
print(f"c2 trained tables: sha256 {sa} / {sb}, final loss {a['trained']['final_loss']}", flush=True)
assert sa == sb, "two training runs in one process differ"
np.savez(out, ent=a["ent"].numpy(), rel=a["rel"].numpy(), sha256=np.array(sa))
print(f"wrote {out}")
