#!/bin/bash
# Round 5, GPU call S: dynamic unit scheduling of the TransE L1 filter sweeps (persistent grid,
# per-XCD-group work counters): L1 / fused-evaluation / sharding tests + the C2 fixture, then C2
# lines with MMRE_SWEEP_DYN=1 (default) / 0 and a 2048-workgroup dynamic grid, the 8-way
# emulation, a C2 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5s
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py tests/test_sweep_filters_gpu.py \
  tests/test_link_gpu.py tests/test_sharding_gloo.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" \
  > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for i in 1; do
  $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_dyn_$i.json 2> $o/c2_dyn_$i.err || exit 1
  MMRE_SWEEP_DYN=0 $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_static_$i.json 2> $o/c2_static_$i.err || exit 1
  MMRE_SWEEP_GRID=2048 $T 300 python -u bench.py --steps 200 --no-cpu-baseline > $o/c2_dyn2048_$i.json 2> $o/c2_dyn2048_$i.err || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8.txt 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_c2.log 2>&1 || exit 1
echo done
