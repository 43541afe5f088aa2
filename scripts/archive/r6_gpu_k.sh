#!/bin/bash
# Round 6, call k: the relation-sharded packing's pair cost after the rescoring aggregation --
# 8-way C2 emulation (all ranks) at pair costs 140 / 90 / 60.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6k
mkdir -p $o
for pc in 140 90 60; do
  MMRE_PAIR_COST=$pc timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu_pc$pc.txt 2>&1 || { tail -20 $o/emu_pc$pc.txt; exit 1; }
  grep -E "^rank|^c2 world" $o/emu_pc$pc.txt | sed "s/^/pc$pc: /" | cut -c1-120
done
echo done
