#!/bin/bash
# round 4, GPU call F: NS model split (DistMult only), relation-row bucket read, L1 counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4f
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_ns_full_gpu.py \
  tests/test_train_gpu.py tests/test_determinism_gpu.py tests/test_sweep_filters_gpu.py > $o/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
for m in transe distmult complex rotate; do
  $T 300 python -u bench.py --config ns --ns-model $m --steps 200 --no-cpu-baseline > $o/bench_ns_$m.json 2> $o/bench_ns_$m.err || exit 1
done
$T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/bench_c2.json 2> $o/bench_c2.err || exit 1
echo done
