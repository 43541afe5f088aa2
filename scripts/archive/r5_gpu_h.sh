#!/bin/bash
# Round 5, GPU call H: per-rank kernel traces at 8-way (rank 7, the slowest) and N = 1 under
# grid-size variants of the sweep (one unit per workgroup vs 2-4) and the gated launches' grid.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5h
mkdir -p $o
T="timeout -k 10"
tr() {  # <name> <args...> : kernel trace of scripts/trace_eval.py
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$n -o run -- python scripts/trace_eval.py "$@" > $o/tr_$n.log 2>&1
}
tr r7 40 world 8 rank 7 || exit 1
MMRE_SWEEP_GRID=2048 tr r7_g2048 40 world 8 rank 7 || exit 1
MMRE_SWEEP_GRID=1536 tr r7_g1536 40 world 8 rank 7 || exit 1
MMRE_SWEEP_GRID=1024 tr r7_g1024 40 world 8 rank 7 || exit 1
MMRE_L1_FB_DIV=16 tr r7_fb16 40 world 8 rank 7 || exit 1
tr n1 40 || exit 1
echo done
