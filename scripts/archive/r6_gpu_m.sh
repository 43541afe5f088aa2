#!/bin/bash
# Round 6, call m: C5 wide-sweep knobs on one box (query tile 128 = two workgroups per CU,
# contiguous ranges instead of windows, grid sizes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6m
mkdir -p $o
bench() {  # <config> <tag> <env...>
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --steps 30 --warmup 5 > $o/${c}_$t.json 2> $o/${c}_$t.err || { tail -20 $o/${c}_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/${c}_$t.json')); print('$c $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3))"
}
bench c5 base MMRE_X=0
bench c5 qt128 MMRE_BF3_QT=128
bench c5 noblk MMRE_BF3_BLOCKED=0
bench c5 base2 MMRE_X=0
echo done
