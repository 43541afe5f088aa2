#!/bin/bash
# Round 5, GPU call E: finalize folded into the gated f32 launch, bf3 64-bit pair counter.
# Fused-path tests + reference fixtures, traces (N = 1, heavy 8-way share), C2/C3/C5 bench
# lines, the 8-way emulation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5e
mkdir -p $o
T="timeout -k 10"
$T 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py \
  tests/test_sweep_filters_gpu.py tests/test_ref_fixture_gpu.py -k "not c4" -s > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
tr() {  # <name> <args...> : kernel trace of scripts/trace_eval.py
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$n -o run -- python scripts/trace_eval.py "$@" > $o/tr_$n.log 2>&1
}
tr fused 50 || exit 1
tr r3 50 world 8 rank 3 || exit 1
$T 400 python -u bench.py --config c3 --steps 20 --no-cpu-baseline > $o/c3.json 2> $o/c3.err || exit 1
$T 600 python -u bench.py --config c5 --steps 5 --no-cpu-baseline > $o/c5.json 2> $o/c5.err || exit 1
for i in 1 2; do
  $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
echo done
