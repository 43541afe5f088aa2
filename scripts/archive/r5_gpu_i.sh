#!/bin/bash
# Round 5, GPU call I: two evaluation slots on two streams (consecutive evaluations overlap).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5i
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_sharding_gloo.py -k "undecided or complex" -s > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
for i in 1 2; do
  $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
  $T 300 python -u bench.py --steps 200 --no-cpu-baseline --eval-streams 1 > $o/c2_s1_$i.json 2> $o/c2_s1_$i.err || exit 1
done
echo done
