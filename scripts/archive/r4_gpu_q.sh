#!/bin/bash
# round 4, GPU call Q: L1 filter tests, C2 bench line, kernel trace of the C2 evaluation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4q
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sweep_filters_gpu.py \
  tests/test_link_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" > $o/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2.json 2> $o/c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof.log 2>&1 || exit 1
echo done
