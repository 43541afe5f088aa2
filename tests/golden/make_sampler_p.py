"""make_sampler_p.py -- golden batches of sampling(..., p=True) from the REFERENCE's Base.so.

The KL-weighted relation corruption (Corrupt.h:111-147, table from importProb, Reader.h:26-49)
is reached only through Base.so's C API (the Python TrainDataLoader never passes p). This script
runs the reference's own C++ core -- oracle/_ref/Base.so, compiled from
/root/reference/OpenKE/openke/base/Base.cpp by oracle/Makefile (the sanctioned compile recipe);
no reference Python is imported -- on a small synthetic dataset written here, dense in relations
per (h, t) pair so the exclusions matter (one pair holds every relation but one, another holds
every relation: its compacted list is empty and the reference returns -1), with a synthetic
kl_prob.txt, and stores the batches and LCG states as tests/golden/sampler_p.npz.

Runs only in the build container. Usage:  python tests/golden/make_sampler_p.py
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DATA = os.path.join(HERE, "data", "prel")


def write_dataset(path, n_ent=40, n_rel=9, seed=3):
    """OpenKE directory format (entity2id / relation2id / train2id "h t r", kl_prob.txt)."""
    rng = np.random.default_rng(seed)
    os.makedirs(path, exist_ok=True)
    trip = set()
    pairs = {(int(h), int(t)) for h, t in rng.integers(0, n_ent, (260, 2)) if h != t}
    for h, t in sorted(pairs):
        k = int(rng.integers(1, n_rel + 1)) if rng.random() < 0.3 else 1
        for r in rng.choice(n_rel, k, replace=False):
            trip.add((h, t, int(r)))
    for r in range(n_rel - 1):  # (0, 1): every relation but the last
        trip.add((0, 1, r))
    for r in range(n_rel):  # (2, 3): every relation
        trip.add((2, 3, r))
    trip = sorted(trip)
    with open(os.path.join(path, "entity2id.txt"), "w") as f:
        f.write(f"{n_ent}\n" + "".join(f"e{i}\t{i}\n" for i in range(n_ent)))
    with open(os.path.join(path, "relation2id.txt"), "w") as f:
        f.write(f"{n_rel}\n" + "".join(f"r{i}\t{i}\n" for i in range(n_rel)))
    with open(os.path.join(path, "train2id.txt"), "w") as f:
        f.write(f"{len(trip)}\n" + "".join(f"{h} {t} {r}\n" for h, t, r in trip))
    for name in ("valid2id.txt", "test2id.txt"):  # one train triple each (the loaders want the files)
        with open(os.path.join(path, name), "w") as f:
            h, t, r = trip[0]
            f.write(f"1\n{h} {t} {r}\n")
    kl = rng.uniform(0.0, 3.0, n_rel * (n_rel - 1))
    with open(os.path.join(path, "kl_prob.txt"), "w") as f:
        f.write(" ".join(f"{x:.6f}" for x in kl) + "\n")


WIDE_REL, WIDE_SEED, WIDE_TEMPS = 200, 11, (0.1, 0.5, 1.0, 2.0)


def wide_kl_text(n_rel=WIDE_REL, seed=WIDE_SEED):
    """kl_prob.txt of a 200-relation table with a wide value range (exp of -x / T spans many
    binades, so a float-vs-double exp would show), regenerated identically by the CPU test."""
    kl = np.random.default_rng(seed).uniform(0.0, 20.0, n_rel * (n_rel - 1))
    return " ".join(f"{x:.6f}" for x in kl) + "\n"


def write_wide(path, n_rel=WIDE_REL):
    """Minimal OpenKE directory with n_rel relations (importProb reads relationTotal and
    kl_prob.txt only)."""
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "entity2id.txt"), "w") as f:
        f.write("2\ne0\t0\ne1\t1\n")
    with open(os.path.join(path, "relation2id.txt"), "w") as f:
        f.write(f"{n_rel}\n" + "".join(f"r{i}\t{i}\n" for i in range(n_rel)))
    for name in ("train2id.txt", "valid2id.txt", "test2id.txt"):
        with open(os.path.join(path, name), "w") as f:
            f.write("1\n0 1 0\n")
    with open(os.path.join(path, "kl_prob.txt"), "w") as f:
        f.write(wide_kl_text(n_rel))


def load_base():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "Base.so"))
    P, I = ctypes.c_void_p, ctypes.c_int64
    lib.setInPath.argtypes = [ctypes.c_char_p]
    lib.setWorkThreads.argtypes = [I]
    lib.setBern.argtypes = [I]
    lib.importProb.argtypes = [ctypes.c_float]
    lib.getTrainTotal.restype = I
    lib.getRelationTotal.restype = I
    lib.sampling.argtypes = [P, P, P, P, I, I, I, I, ctypes.c_bool, ctypes.c_bool, ctypes.c_bool]
    return lib


def seeds_now(lib, threads):
    p = ctypes.c_void_p.in_dll(lib, "next_random").value
    return np.ctypeslib.as_array((ctypes.c_uint64 * threads).from_address(p)).copy()


def main():
    write_dataset(DATA)
    lib = load_base()
    res = {}
    cases = [
        ("t4_b64_k2_r2_bern1_T1", dict(threads=4, B=64, neg=2, negrel=2, mode=0, bern=1, temp=1.0)),
        ("t3_b70_k0_r3_T05", dict(threads=3, B=70, neg=0, negrel=3, mode=0, bern=0, temp=0.5)),
        ("t8_b97_k1_r1_m-1_T2", dict(threads=8, B=97, neg=1, negrel=1, mode=-1, bern=0, temp=2.0)),
        ("t2_b33_k3_r4_m1_T1", dict(threads=2, B=33, neg=3, negrel=4, mode=1, bern=0, temp=1.0)),
    ]
    for name, c in cases:
        lib.setInPath((DATA.rstrip("/") + "/").encode())
        lib.setWorkThreads(c["threads"])
        lib.setBern(c["bern"])
        lib.randReset()
        lib.importTrainFiles()
        lib.importProb(c["temp"])
        res[f"{name}_seeds0"] = seeds_now(lib, c["threads"])
        n = c["B"] * (1 + c["neg"] + c["negrel"])
        for step in range(3):
            bh, bt, br = (np.zeros(n, np.int64) for _ in range(3))
            by = np.zeros(n, np.float32)
            lib.sampling(bh.ctypes.data, bt.ctypes.data, br.ctypes.data, by.ctypes.data, c["B"], c["neg"],
                         c["negrel"], c["mode"], True, True, False)
            res[f"{name}_step{step}"] = np.stack([bh, bt, br]).astype(np.int64)
            res[f"{name}_y{step}"] = by
        res[f"{name}_seeds_end"] = seeds_now(lib, c["threads"])
        res[f"{name}_cfg"] = np.array([c["threads"], c["B"], c["neg"], c["negrel"], c["mode"], c["bern"]], np.int64)
        res[f"{name}_temp"] = np.array(c["temp"], np.float32)
        res[f"{name}_train_total"] = np.array(lib.getTrainTotal(), np.int64)
        # the table the draws came from (Reader.h's global `prob`, n_rel x (n_rel - 1) floats)
        R = int(lib.getRelationTotal())
        p = ctypes.c_void_p.in_dll(lib, "prob").value
        res[f"{name}_prob"] = np.ctypeslib.as_array((ctypes.c_float * (R * (R - 1))).from_address(p)).copy()
    # the prob table alone over 200 relations and a wide KL range (Reader.h:40's
    # unqualified exp(float) is (float)exp((double)x) under libstdc++)
    import tempfile
    wide = tempfile.mkdtemp(prefix="mmre_prel200_")
    write_wide(wide)
    lib.setInPath((wide.rstrip("/") + "/").encode())
    lib.setWorkThreads(1)
    lib.importTrainFiles()
    R = int(lib.getRelationTotal())
    assert R == WIDE_REL
    for T in WIDE_TEMPS:
        lib.importProb(T)
        p = ctypes.c_void_p.in_dll(lib, "prob").value
        res[f"wide_prob_T{T}"] = np.ctypeslib.as_array((ctypes.c_float * (R * (R - 1))).from_address(p)).copy()
    np.savez_compressed(os.path.join(HERE, "sampler_p.npz"), **res)
    neg1 = sum(int((res[k][2] == -1).sum()) for k in res if "_step" in k)
    print("sampler_p fixture:", len(cases), "cases; relation negatives equal to -1 (empty list):", neg1)


if __name__ == "__main__":
    main()
