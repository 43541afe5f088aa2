#!/bin/bash
# Round 6, call s: the wide sweep's DMA cursor with fixed per-lane source offsets and the unit
# map as a template parameter -- filter parity tests, C5 / C3 fixtures, then C5 A/B against the
# final-pass build (abl/head_6882e169.so) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6s
mkdir -p $o
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
$T 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_ref_fixture_gpu.py -k "c5 or c3" > $o/pytest_fix.log 2>&1 || { tail -30 $o/pytest_fix.log; exit 1; }
tail -1 $o/pytest_fix.log
for rep in 1 2; do
for v in head_6882e169 shipped; do
  if [ $v = shipped ]; then L=multimodal-relation-extrapolation_amd/mmre/lib/libmmre_hip.so; else L=abl/$v.so; fi
  MMRE_LIB=$L $T 400 python -u bench.py --config c5 --no-cpu-baseline --steps 30 --warmup 3 > $o/c5_${v}_$rep.json 2> $o/c5_${v}_$rep.err || { tail -20 $o/c5_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$o/c5_${v}_$rep.json'));r=d['roofline'];print('c5 $v',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(r['frac'],3),d['mfma_filter']['undecided_pairs'])"
done
done
echo done
