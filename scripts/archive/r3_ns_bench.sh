#!/bin/bash
# NS step bench + kernel trace (round 3). usage: bash scripts/r3_ns_bench.sh [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=${1:-ns}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config ns --steps 200 --warmup 10 > gpurun_out/r3_bench_$tag.json 2> gpurun_out/r3_bench_$tag.err || exit $?
timeout -k 10 300 python bench.py --config ns --ns-neg 10 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r3_bench_${tag}10.json 2> gpurun_out/r3_bench_${tag}10.err || exit $?
timeout -k 10 300 python bench.py --config ns --ns-prefetch --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r3_bench_${tag}_prefetch.json 2> gpurun_out/r3_bench_${tag}_prefetch.err || exit $?
rm -rf gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --config ns --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r3_prof_$tag.log 2>&1 || exit $?
