#!/bin/bash
# Round 5, GPU call J: K1 two global rounds per query block, K2 rows prefetched + one atomicMax per
# chunk; bit-identity (fused == separate), fixtures, traces (rank 7 of 8, N = 1), bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5j
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py tests/test_sweep_filters_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" -s > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
tr() {  # <name> <args...> : kernel trace of scripts/trace_eval.py
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$n -o run -- python scripts/trace_eval.py "$@" > $o/tr_$n.log 2>&1
}
tr r7 40 world 8 rank 7 || exit 1
tr n1 40 || exit 1
for i in 1 2; do
  $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
done
echo done
