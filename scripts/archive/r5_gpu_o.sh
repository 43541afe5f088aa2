#!/bin/bash
# Round 5, GPU call O: the pipelined TransE training step (mmre_ns_step_openke_pipe): NS / train
# tests + the C2 reference fixture (its tables come from the trainer), then the NS bench line
# (two-launch step) and its kernel trace; the host-loop probe of the 8-way rank 3 share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5o
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ns_full_gpu.py tests/test_train_gpu.py \
  "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
$T 300 python -u bench.py --config ns > $o/bench_ns.json 2> $o/bench_ns.err || { tail -20 $o/bench_ns.err; exit 1; }
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_ns -o run -- \
  python bench.py --config ns --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_ns.log 2>&1 || exit 1
$T 300 python -u scripts/host_loop_probe.py world 8 rank 3 > $o/probe_w8r3.txt 2>&1 || exit 1
$T 300 python -u scripts/host_loop_probe.py world 1 rank 0 > $o/probe_n1.txt 2>&1 || exit 1
echo done
