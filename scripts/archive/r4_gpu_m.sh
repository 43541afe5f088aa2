#!/bin/bash
# round 4, GPU call M: the 8-bit L1 code filter -- filter / C2 fixture / link tests, C2 bench line, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4m
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  tests/test_sweep_filters_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" tests/test_link_gpu.py \
  > $o/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2.json 2> $o/c2.err || exit 1
MMRE_L1_BITS=16 timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_b16.json 2> $o/c2_b16.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof.log 2>&1 || exit 1
echo done
