#!/bin/bash
# Round profiling on the GPU box: kernel-trace stats + PMC passes per config.
# usage: scripts/profile_round.sh <tag> <config...>
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$cfg -o run -- \
      python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${tag}_$cfg.log 2>&1 || exit $?
  scripts/pmc.sh ${tag}_$cfg --config $cfg || exit $?
done
