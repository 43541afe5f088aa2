#!/bin/bash
# Round 5, GPU call Q: the pipelined NS step's A/B (this build; abl/ns_noprep: no pre-pass in the
# row owner; abl/ns_smplast: the sampler workgroups after the row workgroups) -- bench lines +
# kernel traces; the 8-way C2 emulation with pinned staging buffers (the bench's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5q
mkdir -p $o
T="timeout -k 10"
for v in base ns_noprep ns_smplast; do
  if [ $v = base ]; then L=""; else L="MMRE_LIB=$PWD/abl/$v.so"; fi
  env $L $T 300 python -u bench.py --config ns --no-cpu-baseline > $o/ns_$v.json 2> $o/ns_$v.err || exit 1
  env $L $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$v -o run -- \
    python bench.py --config ns --steps 20 --warmup 3 --no-cpu-baseline > $o/tr_$v.log 2>&1 || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
echo done
