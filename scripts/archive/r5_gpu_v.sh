#!/bin/bash
# Round 5, GPU call V: dynamic-scheduling chunk of 4 units (this build) against 8 and 16
# (abl/dyn_ch8, abl/dyn_ch16): C2 lines twice each, the 8-way emulation of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5v
mkdir -p $o
T="timeout -k 10"
for i in 1 2; do
  for v in base dyn_ch8 dyn_ch16; do
    if [ $v = base ]; then L=""; else L="MMRE_LIB=$PWD/abl/$v.so"; fi
    env $L $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_${v}_$i.json 2> $o/c2_${v}_$i.err || exit 1
  done
done
for v in base dyn_ch8 dyn_ch16; do
  if [ $v = base ]; then L=""; else L="MMRE_LIB=$PWD/abl/$v.so"; fi
  env $L $T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8_$v.txt 2>&1 || exit 1
done
echo done
