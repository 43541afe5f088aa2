#!/bin/bash
# Round 5, GPU call C: K1 with atomic accumulators; per-kernel traces of the fused C2 evaluation
# (default, no second rescoring level, separate launches) at N = 1 and for the heavy 8-way
# share; the bf3 sweep's lock-step windows (C3 / C5 bench lines, blocked vs contiguous ranges).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5c
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size" \
  "tests/test_sweep_filters_gpu.py::test_mfma_filter_counts_equal_exact_sweep_and_oracle" -s > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
tr() {  # <name> <args...> : kernel trace of scripts/trace_eval.py
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$n -o run -- python scripts/trace_eval.py "$@" > $o/tr_$n.log 2>&1
}
tr fused 50 || exit 1
MMRE_L1_RESCORE16=0 tr nol2 50 || exit 1
MMRE_FUSED_EVAL=0 tr sep 50 || exit 1
tr r3 50 world 8 rank 3 || exit 1
MMRE_L1_RESCORE16=0 tr r3nol2 50 world 8 rank 3 || exit 1
for c in c3 c5; do
  $T 400 python -u bench.py --config $c --steps 20 --no-cpu-baseline > $o/$c.json 2> $o/$c.err || exit 1
  MMRE_BF3_BLOCKED=0 $T 400 python -u bench.py --config $c --steps 20 --no-cpu-baseline > $o/${c}_ranges.json 2> $o/${c}_ranges.err || exit 1
done
echo done
