#!/bin/bash
# Round 5, GPU call ZB: the wide split-bf16 sweep, second form (k_sweep_bf3w<2, QT>: entity rows
# as the MFMA's A operand, per-lane counts against per-query thresholds; abl/bf3w2.so = the tree
# with it on by default): bf3 filter tests and the C3 / C5 reference fixtures, then C5 / C3 lines
# for QT 256 / 128 and the 128 x 128 sweep (MMRE_BF3_WIDE=0, same library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5zb
mkdir -p $o
T="timeout -k 10"
export MMRE_LIB=abl/bf3w2.so
for qt in 256 128; do
  MMRE_BF3_QT=$qt $T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py -k mfma_filter \
    > $o/pytest_filters_$qt.log 2>&1 || { tail -40 $o/pytest_filters_$qt.log; exit 1; }
  tail -1 $o/pytest_filters_$qt.log
  MMRE_BF3_QT=$qt $T 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_ref_fixture_gpu.py -k "c3 or c5" \
    > $o/pytest_fix_$qt.log 2>&1 || { tail -40 $o/pytest_fix_$qt.log; exit 1; }
  tail -1 $o/pytest_fix_$qt.log
done
for c in c5 c3; do
  for v in "1 256" "1 128" "0 128"; do
    set -- $v
    MMRE_BF3_WIDE=$1 MMRE_BF3_QT=$2 $T 300 python -u bench.py --config $c --no-cpu-baseline > $o/${c}_w$1_$2.json 2> $o/${c}_w$1_$2.err || exit 1
    python -c "import json;d=json.load(open('$o/${c}_w$1_$2.json'));r=d['roofline'];print('$c wide=$1 qt=$2',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(r['frac'],3))"
  done
done
MMRE_BF3_WIDE=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_c5 -o run -- \
  python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --eval-streams 1 > $o/tr_c5.log 2>&1 || exit 1
grep "bf3" $o/tr_c5/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,40), $2}'
echo done
