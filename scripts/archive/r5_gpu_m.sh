#!/bin/bash
# Round 5, GPU call M: per-kernel traces of the fused C2 evaluation (8-way shares of ranks 0 and
# 3, and N = 1), C3 / C5 bench lines (bf3 lock-step XCD windows) with their kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5m
mkdir -p $o
T="timeout -k 10"
tr() {  # <name> <args...> : kernel trace of scripts/trace_eval.py
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$n -o run -- python scripts/trace_eval.py "$@" > $o/tr_$n.log 2>&1
}
tr r3 40 world 8 rank 3 || exit 1
tr r0 40 world 8 rank 0 || exit 1
tr n1 40 || exit 1
for c in c3 c5; do
  $T 400 python -u bench.py --config $c > $o/bench_$c.json 2> $o/bench_$c.err || exit 1
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$c -o run -- \
    python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_$c.log 2>&1 || exit 1
done
echo done
