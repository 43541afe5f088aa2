#!/bin/bash
# Round 6, call q: wide split-bf16 sweep decision pass (branch-free thresholds, a NaN-propagating
# max screen per 16-value block, the unit's first stage from C = 0) -- filter parity tests, then
# C5 A/B against the previous build (abl/head_82df655.so) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6q
mkdir -p $o
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
$T 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_ref_fixture_gpu.py -k "c5 or c3" > $o/pytest_fix.log 2>&1 || { tail -30 $o/pytest_fix.log; exit 1; }
tail -2 $o/pytest_fix.log
for v in shipped head_82df655 shipped head_82df655; do
  if [ $v = shipped ]; then L=multimodal-relation-extrapolation_amd/mmre/lib/libmmre_hip.so; else L=abl/$v.so; fi
  MMRE_LIB=$L $T 400 python -u bench.py --config c5 --no-cpu-baseline --steps 30 --warmup 3 > $o/c5_$v.json 2> $o/c5_$v.err || { tail -20 $o/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/c5_$v.json'));r=d['roofline'];p=d['parity'];print('c5 $v',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(r['frac'],3),p.get('unexplained_mismatches'),d['mfma_filter']['undecided_pairs'])"
done
echo done
