#!/bin/bash
# Round 5, GPU call R: persistent sweep grids with two evaluation streams -- C2 bench lines at
# MMRE_SWEEP_GRID = 512 / 768 / 1024 / 1536 and the default, twice; the 8-way emulation at 512 / 768.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5r
mkdir -p $o
T="timeout -k 10"
for i in 1 2; do
  for g in def 512 768 1024 1536; do
    if [ $g = def ]; then E=""; else E="MMRE_SWEEP_GRID=$g"; fi
    env $E $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_g${g}_$i.json 2> $o/c2_g${g}_$i.err || exit 1
  done
done
for g in 512 768; do
  MMRE_SWEEP_GRID=$g $T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8_g$g.txt 2>&1 || exit 1
done
echo done
