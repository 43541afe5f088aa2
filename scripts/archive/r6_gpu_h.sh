#!/bin/bash
# Round 6, call h: C5 same-box A/B -- the committed build (abl/head_a1.so) against the dynamic
# window order (this tree; MMRE_BF3W_DYN=0 / 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6h
mkdir -p $o
bench() {  # <config> <tag> <env...>
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 5 > $o/${c}_$t.json 2> $o/${c}_$t.err || { tail -20 $o/${c}_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/${c}_$t.json')); print('$c $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3), d['mfma_filter']['undecided_pairs'])"
}
bench c5 head MMRE_LIB=abl/head_a1.so
bench c5 dyn1 MMRE_X=0
bench c5 dyn0 MMRE_BF3W_DYN=0
bench c5 head2 MMRE_LIB=abl/head_a1.so
echo done
