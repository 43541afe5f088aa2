#!/bin/bash
# Round 5, GPU call T: dynamic scheduling with persistent grids below the resident count (room for
# the other evaluation stream): C2 lines at MMRE_SWEEP_GRID = 640 / 768 / 896 and the default
# (1,024), the 8-way emulation at 768 / 896.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5t
mkdir -p $o
T="timeout -k 10"
for i in 1 2; do
  for g in def 640 768 896; do
    if [ $g = def ]; then E=""; else E="MMRE_SWEEP_GRID=$g"; fi
    env $E $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_g${g}_$i.json 2> $o/c2_g${g}_$i.err || exit 1
  done
done
for g in 768 896; do
  MMRE_SWEEP_GRID=$g $T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8_g$g.txt 2>&1 || exit 1
done
echo done
