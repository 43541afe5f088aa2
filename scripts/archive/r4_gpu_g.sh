#!/bin/bash
# round 4, GPU call G: row owner at 7 waves / SIMD, bf3 epilogue for predict = -s
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4g
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_ns_full_gpu.py \
  tests/test_sweep_filters_gpu.py tests/test_link_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c3]" \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c5]" > $o/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
$T 300 python -u bench.py --config ns --steps 200 --no-cpu-baseline > $o/bench_ns_transe.json 2> $o/bench_ns_transe.err || exit 1
for c in c3 c5; do
  $T 300 python -u bench.py --config $c --steps 20 --no-cpu-baseline > $o/bench_$c.json 2> $o/bench_$c.err || exit 1
done
echo done
