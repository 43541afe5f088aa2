#!/bin/bash
# round 4, GPU call A: the changed kernels' tests + smoke + short benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4a
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  tests/test_determinism_gpu.py tests/test_sweep_filters_gpu.py tests/test_ns_full_gpu.py tests/test_train_gpu.py \
  tests/test_api_gpu.py > gpurun_out/r4a/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
$T 300 python -u bench.py --config ns --steps 200 --no-cpu-baseline > gpurun_out/r4a/bench_ns.json 2> gpurun_out/r4a/bench_ns.err || exit 1
$T 300 python -u bench.py --steps 100 --no-cpu-baseline > gpurun_out/r4a/bench_c2.json 2> gpurun_out/r4a/bench_c2.err || exit 1
echo done
