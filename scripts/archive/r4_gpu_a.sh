#!/bin/bash
# round 4, GPU call A: trained C2 tables for the fixture, the changed kernels' tests, smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4a
T="timeout -k 10"
$T 300 python -u scripts/dump_trained_tables.py gpurun_out/trained_c2.npz > gpurun_out/r4a/dump.log 2>&1 || { echo "dump failed"; exit 1; }
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  tests/test_sweep_filters_gpu.py tests/test_determinism_gpu.py tests/test_ns_full_gpu.py tests/test_train_gpu.py \
  tests/test_api_gpu.py tests/test_link_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c3]" \
  > gpurun_out/r4a/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
echo done
