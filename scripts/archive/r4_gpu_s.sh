#!/bin/bash
# round 4, final: per-rank shard emulations (C2 relation- and entity-sharded, C4) on the final build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/final4
mkdir -p $o
rm -f $o/c2_shard_emulation.txt $o/c4_shard_emulation.txt
T="timeout -k 10"
for W in 2 4 8; do
  $T 300 python -u scripts/step_breakdown.py --emulate-world $W --graph --config c2 >> $o/c2_shard_emulation.txt 2>&1 || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --entity --config c2 >> $o/c2_shard_emulation.txt 2>&1 || exit 1
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c4 >> $o/c4_shard_emulation.txt 2>&1 || exit 1
echo done
