#!/bin/bash
# Round 5, GPU call U: dynamic scheduling by chunks of consecutive units (kDynChunk 2 = this build,
# abl/dyn_ch4, abl/dyn_ch1): the fused-evaluation / filter tests on this build, C2 lines at the
# default grid and 768, the 8-way emulation of the chunk-2 build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5u
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py tests/test_sweep_filters_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for v in base dyn_ch4 dyn_ch1; do
  if [ $v = base ]; then L=""; else L="MMRE_LIB=$PWD/abl/$v.so"; fi
  for g in def 768; do
    if [ $g = def ]; then E=""; else E="MMRE_SWEEP_GRID=$g"; fi
    env $L $E $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_${v}_g$g.json 2> $o/c2_${v}_g$g.err || exit 1
  done
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
echo done
