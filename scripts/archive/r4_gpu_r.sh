#!/bin/bash
# round 4, GPU call R: NS tests, NS bench lines (TransE, DistMult), kernel trace of the C2 bench (its trainer's row owner)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4r
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ns_full_gpu.py \
  tests/test_determinism_gpu.py tests/test_train_gpu.py > $o/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest.log; exit 1; }
timeout -k 10 300 python -u bench.py --config ns --steps 200 --no-cpu-baseline > $o/ns.json 2> $o/ns.err || exit 1
timeout -k 10 300 python -u bench.py --config ns --ns-model distmult --steps 200 --no-cpu-baseline > $o/ns_dm.json 2> $o/ns_dm.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $o/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_ns -o run -- python bench.py --config ns --steps 50 --warmup 3 --no-cpu-baseline > $o/prof_ns.log 2>&1 || exit 1
echo done
