#!/bin/bash
# round 4, GPU call H: L1 filter fallback as a gated launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4h
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -s tests/test_sweep_filters_gpu.py \
  tests/test_link_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" > $o/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
$T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/bench_c2.json 2> $o/bench_c2.err || exit 1
MMRE_L1_FILTER=0 $T 300 python -u bench.py --steps 50 --no-cpu-baseline > $o/bench_c2_f32.json 2> $o/bench_c2_f32.err || exit 1
echo done
