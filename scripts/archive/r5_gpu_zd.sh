#!/bin/bash
# Round 5, GPU call ZD: C5 with the wide sweep's 32-column block maxima (k_bf3_enorms): the line,
# and a kernel trace of one-stream evaluations (sweep / norms / split / rescoring times).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5zd
mkdir -p $o
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py -k mfma_filter \
  > $o/pytest_filters.log 2>&1 || { tail -40 $o/pytest_filters.log; exit 1; }
tail -1 $o/pytest_filters.log
$T 400 python -u bench.py --config c5 --no-cpu-baseline > $o/bench_c5.json 2> $o/bench_c5.err || exit 1
python -c "import json;d=json.load(open('$o/bench_c5.json'));r=d['roofline'];print('c5',round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3))"
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_c5 -o run -- \
  python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --eval-streams 1 > $o/tr_c5.log 2>&1 || exit 1
grep "bf3" $o/tr_c5/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,40), $2}'
echo done
