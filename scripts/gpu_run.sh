#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first crash/timeout
# (exit >= 124 or signal), but continue past ordinary test failures (exit 1).
# usage: scripts/gpu_run.sh "<name> <timeout_s> <cmd...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
  name=${spec%% *}; rest=${spec#* }; to=${rest%% *}; cmd=${rest#* }
  echo "=== $name (timeout ${to}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping: $name crashed or timed out"; exit $rc
  fi
  [ $rc -ne 0 ] && status=$rc
done
exit $status
