#!/bin/bash
# Round-3 extra lines on the final build: the NS drop-in path, and the SURVEY 8(f) rows (zsl, gan, m3ae).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/final
mkdir -p $o
timeout -k 10 300 python bench.py --config ns --ns-autograd --no-cpu-baseline > $o/bench_ns_autograd.json 2> $o/bench_ns_autograd.err || exit $?
for c in zsl gan m3ae; do
  timeout -k 10 400 python bench.py --config $c > $o/bench_$c.json 2> $o/bench_$c.err || exit $?
done
