#!/bin/bash
# round 4, GPU call B: the NS tests (two-launch step), bench lines of every config touched this
# round, per-rank shard emulations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s tests/test_ns_full_gpu.py \
  tests/test_train_gpu.py tests/test_determinism_gpu.py > gpurun_out/r4b/pytest_ns.log 2>&1 || { echo "pytest failed"; exit 1; }
for m in transe distmult complex rotate; do
  $T 300 python -u bench.py --config ns --ns-model $m --steps 200 --no-cpu-baseline > gpurun_out/r4b/bench_ns_$m.json 2> gpurun_out/r4b/bench_ns_$m.err || exit 1
done
MMRE_NS_STEP2=0 $T 300 python -u bench.py --config ns --steps 200 --no-cpu-baseline > gpurun_out/r4b/bench_ns_transe_3launch.json 2> gpurun_out/r4b/bench_ns_transe_3launch.err || exit 1
for c in c3 c5 c4; do
  $T 300 python -u bench.py --config $c --steps 20 --no-cpu-baseline > gpurun_out/r4b/bench_$c.json 2> gpurun_out/r4b/bench_$c.err || exit 1
done
$T 300 python -u bench.py --steps 100 --no-cpu-baseline > gpurun_out/r4b/bench_c2.json 2> gpurun_out/r4b/bench_c2.err || exit 1
for W in 2 4 8; do
  $T 300 python -u scripts/step_breakdown.py --emulate-world $W --graph --config c2 >> gpurun_out/r4b/c2_shard_emulation.txt 2>&1 || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --entity --config c2 >> gpurun_out/r4b/c2_shard_emulation.txt 2>&1 || exit 1
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c4 >> gpurun_out/r4b/c4_shard_emulation.txt 2>&1 || exit 1
echo done
