#!/bin/bash
# Round 6, call n: C3 split-bf16 sweep grid / variant A/B after the segmented pair lists
# (one persistent round vs 2-3 rounds of equal ranges; the wide sweep; lock-step windows).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6n
mkdir -p $o
bench() {  # <config> <tag> <env...>
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > $o/${c}_$t.json 2> $o/${c}_$t.err || { tail -20 $o/${c}_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/${c}_$t.json')); print('$c $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3))"
}
bench c3 base MMRE_X=0
bench c3 g768 MMRE_SWEEP_GRID=768
bench c3 g1536 MMRE_SWEEP_GRID=1536
bench c3 g2304 MMRE_SWEEP_GRID=2304
bench c3 g3072 MMRE_SWEEP_GRID=3072
bench c3 wide MMRE_BF3_WIDE=1
bench c3 wide128 MMRE_BF3_WIDE=1 MMRE_BF3_QT=128
bench c3 blk MMRE_BF3_BLOCKED=1
bench c3 base2 MMRE_X=0
echo done
