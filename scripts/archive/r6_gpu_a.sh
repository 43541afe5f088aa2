#!/bin/bash
# Round 6, call a: the review fixes' GPU tests + an 8-way C2 rank-share kernel timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6a
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_ns_full_gpu.py::test_pipelined_train_step_falls_back_when_its_prefetch_is_stale" \
  tests/test_api_gpu.py tests/test_eval_fused_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
timeout -k 10 400 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || { tail -20 $o/emu8.txt; exit 1; }
cat $o/emu8.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $o/tl -o run -- \
  python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 --ranks 1,3 --no-n1 --reps 20 > $o/tl.log 2>&1 || { tail -20 $o/tl.log; exit 1; }
tail -3 $o/tl.log
echo done
