#!/bin/bash
# Interleaved A/B of the sweep kernels on one box: the in-tree library (default, and 16-row MFMA
# K stages via MMRE_MFMA_STAGE=16) against another build (MMRE_LIB), alternating runs.
# usage: scripts/ab_libs.sh <other.so> [configs...]
other=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${@:-c2 c3 c5}; do
  for rep in 1 2; do
    MMRE_LIB=$other TAG=other timeout -k 10 200 python scripts/ab_sweep.py $c 10 2>&1 | grep sweep || exit 1
    TAG=new timeout -k 10 200 python scripts/ab_sweep.py $c 10 2>&1 | grep sweep || exit 1
    [ $c != c2 ] && [ $c != c4 ] && { MMRE_MFMA_STAGE=16 TAG=new_ks16 timeout -k 10 200 python scripts/ab_sweep.py $c 10 2>&1 | grep sweep || exit 1; }
  done
done
