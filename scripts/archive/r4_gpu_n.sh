#!/bin/bash
# round 4, GPU call N: C2 A/B -- 8-bit codes (auto), forced 16-bit, 8-bit with the rescoring skipped (timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4n
mkdir -p $o
T="timeout -k 10 300"
for i in 1 2; do
  $T python -u bench.py --steps 100 --no-cpu-baseline > $o/auto_$i.json 2> $o/auto_$i.err || exit 1
  MMRE_L1_BITS=16 $T python -u bench.py --steps 100 --no-cpu-baseline > $o/b16_$i.json 2> $o/b16_$i.err || exit 1
  MMRE_LIB=$PWD/abl/norescore.so $T python -u bench.py --steps 100 --no-cpu-baseline > $o/norescore_$i.json 2> $o/norescore_$i.err || exit 1
done
echo done
