#!/bin/bash
# Round 5, GPU call Y: the one-call pipelined step for DistMult / ComplEx / RotatE
# (mmre_ns_step_openke_gen_pipe): NS tests, then the NS lines of every model and their traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5y
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ns_full_gpu.py tests/test_train_gpu.py \
  tests/test_api_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for m in transe distmult complex rotate; do
  $T 300 python -u bench.py --config ns --ns-model $m --no-cpu-baseline > $o/ns_$m.json 2> $o/ns_$m.err || exit 1
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$m -o run -- \
    python bench.py --config ns --ns-model $m --steps 20 --warmup 3 --no-cpu-baseline > $o/tr_$m.log 2>&1 || exit 1
done
echo done
