#!/bin/bash
# Round 5, GPU call P: bf3 sweep A/B (MMRE_BF3_BLOCKED=1 lock-step XCD windows vs 0 contiguous
# unit ranges) on C3 and C5, twice each, bench lines without the CPU leg; C2 8-way emulation grids.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5p
mkdir -p $o
T="timeout -k 10"
for i in 1 2; do
  for c in c3 c5; do
    for b in 1 0; do
      MMRE_BF3_BLOCKED=$b $T 300 python -u bench.py --config $c --steps 50 --no-cpu-baseline > $o/${c}_b${b}_$i.json 2> $o/${c}_b${b}_$i.err || exit 1
    done
  done
done
# the 8-way C2 emulation with persistent sweep grids (MMRE_SWEEP_GRID = workgroups) against the
# default one-unit-per-workgroup grid of a rank's share
for g in 1024 2048 3072; do
  MMRE_SWEEP_GRID=$g $T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8_g$g.txt 2>&1 || exit 1
done
echo done
