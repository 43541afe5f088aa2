#!/bin/bash
# round 4, GPU call V: the quantization kernel's grid / unroll -- L1 tests, C2 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4v
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sweep_filters_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" > $o/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof.log 2>&1 || exit 1
echo done
