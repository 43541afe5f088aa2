#!/bin/bash
# Round 5, GPU call A: the C2 sweep without scratch spills (one-pass integer epilogue, per-tile
# values recomputed from opaque copies), the rescoring guard, wide-row backward, the fused TransE
# L1 evaluation (mmre_link_evaluate_l1q).
#   targeted -m gpu tests; C2 bench lines: this build, MMRE_FUSED_EVAL=0 (separate launches),
#   abl/kku1.so (the 8-bit loop at one LDS row per iteration); 8-way relation-sharded emulation
#   fused and separate; a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5a
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py \
  tests/test_link_gpu.py tests/test_sweep_filters_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" \
  tests/test_wide_rows_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for i in 1 2; do
  $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
  MMRE_FUSED_EVAL=0 $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/sep_$i.json 2> $o/sep_$i.err || exit 1
  MMRE_LIB=$PWD/abl/kku1.so MMRE_FUSED_EVAL=0 $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/kku1_$i.json 2> $o/kku1_$i.err || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
MMRE_FUSED_EVAL=0 $T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8_sep.txt 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_c2.log 2>&1 || exit 1
echo done
