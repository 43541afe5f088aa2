#!/bin/bash
# Round 6, call g: the wide sweep's dynamic window order (tests, C5 A/B, C5 PMC traffic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6g
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_sweep_filters_gpu.py -k "wide or mfma" > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
bench() {  # <config> <tag> <env...>
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 5 > $o/${c}_$t.json 2> $o/${c}_$t.err || { tail -20 $o/${c}_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/${c}_$t.json')); print('$c $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3), d['mfma_filter']['undecided_pairs'])"
}
bench c5 dyn1 MMRE_X=0
bench c5 dyn0 MMRE_BF3W_DYN=0
bench c5 dyn1b MMRE_X=0
# FETCH / WRITE of the wide sweep per launch, both orders
for v in 1 0; do
  MMRE_BF3W_DYN=$v timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc_f$v -o run -- python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $o/pmc_f$v.log 2>&1 || { tail -5 $o/pmc_f$v.log; exit 1; }
  MMRE_BF3W_DYN=$v timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $o/pmc_h$v -o run -- python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $o/pmc_h$v.log 2>&1 || { tail -5 $o/pmc_h$v.log; exit 1; }
done
echo done
