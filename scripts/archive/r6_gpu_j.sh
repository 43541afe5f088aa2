#!/bin/bash
# Round 6, call j: per-query aggregation of the L1 rescoring's count atomics -- L1 tests, C2
# reference fixture, C2 same-box A/B against the committed build (abl/head_a1.so), 8-way shares.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6j
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_sweep_filters_gpu.py tests/test_eval_fused_gpu.py tests/test_link_gpu.py "tests/test_ref_fixture_gpu.py" > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
bench() {  # <config> <tag> <env...>
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --steps 200 --warmup 10 > $o/${c}_$t.json 2> $o/${c}_$t.err || { tail -20 $o/${c}_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/${c}_$t.json')); print('$c $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3))"
}
bench c2 new MMRE_X=0
bench c2 head MMRE_LIB=abl/head_a1.so
bench c2 new2 MMRE_X=0
bench c2 head2 MMRE_LIB=abl/head_a1.so
for t in new head; do
  lib=""; [ $t = head ] && lib=abl/head_a1.so
  MMRE_LIB=$lib timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 --ranks 1,3,7 > $o/emu_$t.txt 2>&1 || { tail -20 $o/emu_$t.txt; exit 1; }
  grep -E "^N=1|^rank" $o/emu_$t.txt | sed "s/^/$t: /" | cut -c1-150
done
echo done
