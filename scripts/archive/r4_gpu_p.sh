#!/bin/bash
# round 4, GPU call P: C2 A/B -- the software-pipelined L1 inner loop vs the plain one (abl/nopipe.so), L1 filter tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4p
mkdir -p $o
T="timeout -k 10 300"
for i in 1 2; do
  $T python -u bench.py --steps 100 --no-cpu-baseline > $o/pipe_$i.json 2> $o/pipe_$i.err || exit 1
  MMRE_LIB=$PWD/abl/nopipe.so $T python -u bench.py --steps 100 --no-cpu-baseline > $o/nopipe_$i.json 2> $o/nopipe_$i.err || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sweep_filters_gpu.py \
  tests/test_link_gpu.py > $o/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest.log; exit 1; }
echo done
