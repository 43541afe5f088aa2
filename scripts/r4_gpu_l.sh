#!/bin/bash
# round 4, GPU call L: C2 A/B on one box -- this build vs the round-3 tree (ab_r3, a git worktree at db688e2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r4l
mkdir -p $o
T="timeout -k 10 300"
for i in 1 2; do
  $T python -u bench.py --steps 200 --no-cpu-baseline > $o/cur_$i.json 2> $o/cur_$i.err || exit 1
  (cd ab_r3 && $T python -u bench.py --steps 200 --no-cpu-baseline) > $o/r3_$i.json 2> $o/r3_$i.err || exit 1
done
$T rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_cur -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_cur.log 2>&1 || exit 1
cd ab_r3 && $T rocprofv3 --kernel-trace --stats --output-format csv -d ../$o/prof_r3 -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > ../$o/prof_r3.log 2>&1 || exit 1
echo done
