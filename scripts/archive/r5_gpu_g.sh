#!/bin/bash
# Round 5, GPU call G: heavy queries spread over the query tiles (rank_order "spread") vs Test.h order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5g
mkdir -p $o
T="timeout -k 10"
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
$T 300 python -u scripts/step_breakdown.py --emulate-world 4 --graph --config c2 > $o/emu4.txt 2>&1 || exit 1
$T 300 python -u scripts/step_breakdown.py --emulate-world 2 --graph --config c2 > $o/emu2.txt 2>&1 || exit 1
for i in 1 2; do
  $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
  $T 300 python -u bench.py --steps 100 --no-cpu-baseline --pack count > $o/c2_count_$i.json 2> $o/c2_count_$i.err || exit 1
done
echo done
