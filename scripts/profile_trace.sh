#!/bin/bash
# Kernel-trace summaries of the bench workloads with enough timed steps that warmup launches
# do not dominate the averages. usage: scripts/profile_trace.sh <tag> <steps> <config...>
tag=$1; steps=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$cfg -o run -- \
      python bench.py --config $cfg --steps $steps --warmup 3 --no-cpu-baseline > gpurun_out/prof_${tag}_$cfg.log 2>&1 || exit $?
  echo "$cfg traced"
done
