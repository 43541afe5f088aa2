#!/bin/bash
# round 4, GPU call I: C2 kernel trace (where the 1.85 ms goes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4i
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- \
    python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c4 -o run -- \
    python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $o/prof_c4.log 2>&1 || exit 1
echo done
