#!/bin/bash
# Round 6, call b: 8-way C2 rank shares under sweep-grid variants (residency left for the other
# stream's prologue) and chunk sizes; N = 1 under the same variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${R6B_OUT:-r6b}
mkdir -p $o
run() {  # <tag> <env...>
  local t=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 --ranks 1,3,7 > $o/emu_$t.txt 2>&1 || { tail -20 $o/emu_$t.txt; exit 1; }
  grep -E "^N=1|^rank" $o/emu_$t.txt | sed "s/^/$t: /" | cut -c1-200
}
run base MMRE_X=0
run g8192 MMRE_SWEEP_GRID=8192
run g4096 MMRE_SWEEP_GRID=4096
run g2048 MMRE_SWEEP_GRID=2048

echo done
