#!/bin/bash
# Round 5, GPU call D: fused evaluation without same-address atomic chains (K1 plain partials
# reduced in K2, K3 a wave per group / 128 probe blocks), no second rescoring level; traces at
# N = 1 and the heavy 8-way share; the bf3 regression hunt (C3: this build, the select-based row
# counts, the unsaturated pair counter).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5d
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" -s > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
tr() {  # <name> <args...> : kernel trace of scripts/trace_eval.py
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$n -o run -- python scripts/trace_eval.py "$@" > $o/tr_$n.log 2>&1
}
tr fused 50 || exit 1
MMRE_FUSED_EVAL=0 tr sep 50 || exit 1
tr r3 50 world 8 rank 3 || exit 1
MMRE_FUSED_EVAL=0 tr r3sep 50 world 8 rank 3 || exit 1
for v in "" bf3_select bf3_nosat; do
  lib=${v:+$PWD/abl/$v.so}
  MMRE_LIB=$lib $T 400 python -u bench.py --config c3 --steps 20 --no-cpu-baseline > $o/c3_${v:-cur}.json 2> $o/c3_${v:-cur}.err || exit 1
done
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_c3 -o run -- python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $o/tr_c3.log 2>&1 || exit 1
for i in 1 2; do
  $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
echo done
