#!/bin/bash
# Round 5, GPU call Z: the wide split-bf16 sweep (k_sweep_bf3w, abl/bf3w.so = the tree with the
# wide sweep on by default): bf3 filter tests and the C3 / C5 reference fixtures on it, then
# C5 / C3 lines wide vs 128 x 128 (MMRE_BF3_WIDE=0, same library) and a kernel trace of C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5z
mkdir -p $o
T="timeout -k 10"
export MMRE_LIB=abl/bf3w.so
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py -k mfma_filter \
  > $o/pytest_filters.log 2>&1 || { tail -40 $o/pytest_filters.log; exit 1; }
tail -2 $o/pytest_filters.log
$T 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_ref_fixture_gpu.py -k "c3 or c5" \
  > $o/pytest_fix.log 2>&1 || { tail -40 $o/pytest_fix.log; exit 1; }
tail -2 $o/pytest_fix.log
for c in c5 c3; do
  for w in 1 0; do
    MMRE_BF3_WIDE=$w $T 300 python -u bench.py --config $c --no-cpu-baseline > $o/${c}_w$w.json 2> $o/${c}_w$w.err || exit 1
    python -c "import json;d=json.load(open('$o/${c}_w$w.json'));print('$c wide=$w',d['ms_per_step'],d['roofline'])"
  done
done
MMRE_BF3_WIDE=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_c5 -o run -- \
  python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $o/tr_c5.log 2>&1 || exit 1
grep -i "bf3" $o/tr_c5/run_kernel_stats.csv | cut -c1-200
echo done
