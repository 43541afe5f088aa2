#!/bin/bash
# Round 6, call d: the DistMult raw-row split (filter tests + C5 A/B) and the balanced small-share
# grid (8-way C2 A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6d
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_sweep_filters_gpu.py tests/test_link_gpu.py tests/test_ns_full_gpu.py tests/test_api_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
run() {  # <tag> <env...>
  local t=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 --ranks 1,3,7 > $o/emu_$t.txt 2>&1 || { tail -20 $o/emu_$t.txt; exit 1; }
  grep -E "^N=1|^rank" $o/emu_$t.txt | sed "s/^/$t: /" | cut -c1-190
}
run bal1 MMRE_SWEEP_BALANCE=1
run bal0 MMRE_SWEEP_BALANCE=0
run bal1b MMRE_SWEEP_BALANCE=1
run g8192 MMRE_SWEEP_GRID=8192
for v in 1 0; do
  MMRE_BF3_RAW=$v timeout -k 10 500 python bench.py --config c5 --no-cpu-baseline --steps 30 --warmup 5 > $o/c5_raw$v.json 2> $o/c5_raw$v.err || { tail -20 $o/c5_raw$v.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c5_raw$v.json')); print('c5 raw=$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['mfma_filter'])"
done
c3() {  # <tag> <env...>
  local t=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 100 --warmup 10 > $o/c3_$t.json 2> $o/c3_$t.err || { tail -20 $o/c3_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c3_$t.json')); print('c3 $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['mfma_filter']['undecided_pairs'])"
}
c3 base MMRE_X=0
c3 noepi MMRE_LIB=abl/bf3_noepi.so
c3 emajor MMRE_MFMA_EMAJOR=1
c3 g512 MMRE_SWEEP_GRID=512
c3 g1536 MMRE_SWEEP_GRID=1536
c3 blocked MMRE_BF3_BLOCKED=1
c3 base2 MMRE_X=0
timeout -k 10 500 python bench.py --config c2 --type-constrain --steps 50 --warmup 5 > $o/c2_tc.json 2> $o/c2_tc.err || { tail -20 $o/c2_tc.err; exit 1; }
python -c "import json; d=json.load(open('$o/c2_tc.json')); print('c2 tc', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'], d['parity'])"
echo done
