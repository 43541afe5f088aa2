#!/bin/bash
# Round 5, GPU call N: PMC passes (scripts/pmc.sh) of C2, C3 and C5 on this build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r5n
mkdir -p $o
for c in c2 c3 c5; do bash scripts/pmc.sh r5_$c --config $c > $o/pmc_$c.txt 2>&1 || exit 1; done
echo done
