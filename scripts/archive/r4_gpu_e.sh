#!/bin/bash
# round 4, GPU call E: bf3 KB=2 A/B, generic NS traces, C2 bench (l1 stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4e
mkdir -p $o
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  "tests/test_sweep_filters_gpu.py::test_mfma_filter_counts_equal_exact_sweep_and_oracle" > $o/pytest_kb1.log 2>&1 || { echo "pytest failed"; exit 1; }
MMRE_BF3_KB=2 $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  "tests/test_sweep_filters_gpu.py::test_mfma_filter_counts_equal_exact_sweep_and_oracle" > $o/pytest_kb2.log 2>&1 || { echo "pytest kb2 failed"; exit 1; }
for c in c3 c5; do
  MMRE_BF3_KB=2 $T 300 python -u bench.py --config $c --steps 20 --no-cpu-baseline > $o/bench_${c}_kb2.json 2> $o/bench_${c}_kb2.err || exit 1
done
trace() {  # <name> <bench args...>
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$n -o run -- \
    python bench.py "$@" --warmup 3 --no-cpu-baseline > $o/prof_$n.log 2>&1
}
trace ns_complex --config ns --ns-model complex --steps 50 || exit 1
trace ns_rotate --config ns --ns-model rotate --steps 50 || exit 1
$T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/bench_c2.json 2> $o/bench_c2.err || exit 1
echo done
