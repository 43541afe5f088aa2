#!/bin/bash
# Round 5, GPU call N: PMC passes (scripts/pmc.sh, one counter group per rocprofv3 run) of C2,
# C3, C5 and the NS step on this build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5n
mkdir -p $o
for c in c2 c5 c3 ns; do bash scripts/pmc.sh r5_$c --config $c > $o/pmc_$c.txt 2>&1 || { tail -20 $o/pmc_$c.txt; exit 1; }; done
echo done
