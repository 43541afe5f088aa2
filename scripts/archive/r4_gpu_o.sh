#!/bin/bash
# round 4, GPU call O: PMC passes of the C2 evaluation with 8-bit codes (auto) and forced 16-bit codes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/pmc.sh c2_b8 || exit 1
MMRE_L1_BITS=16 bash scripts/pmc.sh c2_b16 || exit 1
echo done
