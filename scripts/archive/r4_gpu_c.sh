#!/bin/bash
# round 4, GPU call C: L1 stats diagnostic, kernel traces of the NS steps and C3, the reference
# fixtures C2 / C4 / C5 on the production path
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4c
mkdir -p $o
T="timeout -k 10"
$T 300 python -u scripts/probe_l1q_stats.py > $o/probe_l1q.log 2>&1 || { echo "probe failed"; exit 1; }
trace() {  # <name> <bench args...>
  local n=$1; shift
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$n -o run -- \
    python bench.py "$@" --warmup 3 --no-cpu-baseline > $o/prof_$n.log 2>&1
}
trace ns2 --config ns --steps 50 || exit 1
MMRE_NS_STEP2=0 trace ns3 --config ns --steps 50 || exit 1
trace ns_distmult --config ns --ns-model distmult --steps 50 || exit 1
trace c3 --config c3 --steps 20 || exit 1
trace c5 --config c5 --steps 5 || exit 1
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -s tests/test_ref_fixture_gpu.py \
  > $o/pytest_ref.log 2>&1 || { echo "pytest failed"; exit 1; }
echo done
