#!/bin/bash
# RotatE sweep check: parity tests (fast filter, link, reference fixture C4), then the C4 bench
# and a kernel trace of it.
set -o pipefail
tag=${1:-rot}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rotate_filter_gpu.py \
  tests/test_link_gpu.py "tests/test_ref_fixture_gpu.py" > gpurun_out/r3_${tag}_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/r3_bench_c4_$tag.json \
  2> gpurun_out/r3_bench_c4_$tag.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_$tag -- \
  python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r3_prof_c4_$tag.log 2>&1
