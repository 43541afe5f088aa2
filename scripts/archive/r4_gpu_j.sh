#!/bin/bash
# round 4, GPU call J: fallback-flag latency hidden, gated launches one residency round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4${R4TAG:-j}
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -s tests/test_sweep_filters_gpu.py \
  "tests/test_ref_fixture_gpu.py" > $o/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
$T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/bench_c2.json 2> $o/bench_c2.err || exit 1
$T 300 python -u bench.py --config c3 --steps 50 --no-cpu-baseline > $o/bench_c3.json 2> $o/bench_c3.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- \
    python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --train-steps 0 > $o/prof_c2.log 2>&1 || exit 1
echo done
