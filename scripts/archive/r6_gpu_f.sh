#!/bin/bash
# Round 6, call f: segmented bf3 pair lists + the entity-rows-as-A sweep (k_sweep_bf3t): filter
# tests, C3 / C5 reference fixtures, C3 / C5 timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6f
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_sweep_filters_gpu.py tests/test_ref_fixture_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
bench() {  # <config> <tag> <env...>
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --steps 60 --warmup 5 > $o/${c}_$t.json 2> $o/${c}_$t.err || { tail -20 $o/${c}_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/${c}_$t.json')); print('$c $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3), d['mfma_filter']['undecided_pairs'])"
}
bench c3 t1 MMRE_X=0
bench c3 t0 MMRE_BF3_T=0
bench c3 t1_g512 MMRE_SWEEP_GRID=512
bench c5 seg MMRE_X=0
bench c3 t1b MMRE_X=0
echo done
