#!/bin/bash
# Round 5, GPU call X: the bf3 sweep's mask-logic epilogue (compares as wave masks, decisions on
# the scalar unit): the MFMA-filter tests + C3 / C5 reference fixtures, C3 / C5 lines, one PMC
# pass of the C5 sweep's VALU instruction count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5x
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_sweep_filters_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c3]" "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c5]" \
  > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for c in c3 c5; do
  $T 300 python -u bench.py --config $c --steps 50 --no-cpu-baseline > $o/$c.json 2> $o/$c.err || exit 1
done
$T 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $o/pmc_c5 -o run -- \
  python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $o/pmc_c5.log 2>&1 || exit 1
echo done
