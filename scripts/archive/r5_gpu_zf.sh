#!/bin/bash
# Round 5, GPU call ZF: the wide sweep with one barrier per two 16-k stages (four stage buffers;
# abl/bf3pair.so = the tree built with W3_PAIR=1) against the shipped build, on one box:
# MFMA-filter tests and the C5 fixture on the variant, C5 lines of both, a trace of the variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5zf
mkdir -p $o
T="timeout -k 10"
MMRE_LIB=abl/bf3pair.so $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py -k mfma_filter \
  > $o/pytest_filters.log 2>&1 || { tail -40 $o/pytest_filters.log; exit 1; }
tail -1 $o/pytest_filters.log
MMRE_LIB=abl/bf3pair.so $T 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_ref_fixture_gpu.py -k c5 \
  > $o/pytest_fix.log 2>&1 || { tail -40 $o/pytest_fix.log; exit 1; }
tail -1 $o/pytest_fix.log
for v in shipped bf3pair shipped bf3pair; do
  if [ $v = shipped ]; then L=multimodal-relation-extrapolation_amd/mmre/lib/libmmre_hip.so; else L=abl/$v.so; fi
  MMRE_LIB=$L $T 400 python -u bench.py --config c5 --no-cpu-baseline > $o/c5_$v.json 2> $o/c5_$v.err || exit 1
  python -c "import json;d=json.load(open('$o/c5_$v.json'));r=d['roofline'];print('c5 $v',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(r['frac'],3))"
done
MMRE_LIB=abl/bf3pair.so $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_c5 -o run -- \
  python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --eval-streams 1 > $o/tr_c5.log 2>&1 || exit 1
grep "bf3w" $o/tr_c5/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,40), $2}'
echo done
