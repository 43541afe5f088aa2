#!/bin/bash
# Round 6, call e: the entity-rows-as-A bf3 sweep (k_sweep_bf3t) -- filter tests, C3 reference
# fixture, C3 A/B against k_sweep_bf3 (MMRE_BF3_T=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6e
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_sweep_filters_gpu.py -k mfma tests/test_ref_fixture_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
c3() {  # <tag> <env...>
  local t=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 100 --warmup 10 > $o/c3_$t.json 2> $o/c3_$t.err || { tail -20 $o/c3_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c3_$t.json')); print('c3 $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3), d['mfma_filter']['undecided_pairs'])"
}
c3 t1 MMRE_X=0
c3 t0 MMRE_BF3_T=0
c3 t1_g512 MMRE_SWEEP_GRID=512
c3 t1_blk MMRE_BF3_BLOCKED=1
c3 t1_blk512 MMRE_BF3_BLOCKED=1 MMRE_SWEEP_GRID=512
c3 t1b MMRE_X=0
echo done
