#!/bin/bash
# round 4, GPU call T: the widened code-width probe -- L1 tests, 8-way C2 emulation with the per-rank filter record, C2 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4t
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_sweep_filters_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" > $o/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest.log; exit 1; }
timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2.json 2> $o/c2.err || exit 1
echo done
