#!/bin/bash
# Link-sweep check: filter + link + sharding + reference-fixture parity tests, then benches of the
# given configs (default c2) with a kernel trace of each.
set -o pipefail
tag=${1:-sweep}; shift
configs=${@:-c2}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py \
  tests/test_link_gpu.py tests/test_ref_fixture_gpu.py tests/test_sharding_gloo.py -m gpu \
  > gpurun_out/r3_${tag}_tests.log 2>&1 || exit $?
export TMPDIR=/tmp
for c in $configs; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/r3_bench_${c}_$tag.json 2> gpurun_out/r3_bench_${c}_$tag.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${c}_$tag -- \
    python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r3_prof_${c}_$tag.log 2>&1 || exit $?
done
