#!/bin/bash
# Stall / MFMA-utilisation counter passes for an MFMA kernel (one counter group per rocprofv3
# run, no tracing domains combined with --pmc). usage: scripts/pmc_mfma.sh <tag> [bench args...]
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $out/p$i.log; exit $rc; fi
done
