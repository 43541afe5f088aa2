#!/bin/bash
# round 4, GPU call D: owner hub scan fix + parallel bf3 split: tests, L1 stats probe, traces, benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4d
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -s tests/test_sweep_filters_gpu.py \
  tests/test_ns_full_gpu.py tests/test_train_gpu.py tests/test_determinism_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c3]" \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c5]" > $o/pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
$T 300 python -u scripts/probe_l1q_stats.py > $o/probe_l1q.log 2>&1 || { echo "probe failed"; exit 1; }
trace() {  # <name> <bench args...>
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$n -o run -- \
    python bench.py "$@" --warmup 3 --no-cpu-baseline > $o/prof_$n.log 2>&1
}
trace ns --config ns --steps 50 || exit 1
trace c3 --config c3 --steps 20 || exit 1
for m in transe distmult complex rotate; do
  $T 300 python -u bench.py --config ns --ns-model $m --steps 200 --no-cpu-baseline > $o/bench_ns_$m.json 2> $o/bench_ns_$m.err || exit 1
done
for c in c3 c5; do
  $T 300 python -u bench.py --config $c --steps 20 --no-cpu-baseline > $o/bench_$c.json 2> $o/bench_$c.err || exit 1
done
echo done
