#!/bin/bash
# C3 MFMA sweep time vs persistent grid size (MMRE_SWEEP_GRID), interleaved, default last.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for g in 512 768 1024 1536 2048 default; do
    if [ $g = default ]; then E=; else E=$g; fi
    MMRE_SWEEP_GRID=$E TAG=g$g timeout -k 10 200 python scripts/ab_sweep.py ${1:-c3} 10 2>&1 | grep sweep || exit 1
  done
done
