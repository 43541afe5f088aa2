#!/bin/bash
# Round 5, GPU call W: dynamic scheduling with the chunk picked per launch (4 units per claim when
# a workgroup sweeps >= 16 units, else 1): tests (fused evaluation, filters, sharding, the C2 and
# the widened C4 reference fixtures), C2 lines, the 2 / 4 / 8-way emulation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5w
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_eval_fused_gpu.py tests/test_sweep_filters_gpu.py \
  tests/test_sharding_gloo.py tests/test_ref_fixture_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for i in 1 2; do
  $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
done
for w in 2 4 8; do
  $T 300 python -u scripts/step_breakdown.py --emulate-world $w --graph --config c2 > $o/emu$w.txt 2>&1 || exit 1
done
echo done
