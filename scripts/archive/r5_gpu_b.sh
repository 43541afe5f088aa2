#!/bin/bash
# Round 5, GPU call B: the fused evaluation without fences (sc1 hand-off), the 16-bit second
# rescoring level, cost-packed sharding.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5b
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_fused_gpu.py \
  tests/test_link_gpu.py tests/test_sweep_filters_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" \
  tests/test_sharding_gloo.py -s > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for i in 1 2; do
  $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/c2_$i.json 2> $o/c2_$i.err || exit 1
  MMRE_L1_RESCORE16=0 $T 300 python -u bench.py --steps 100 --no-cpu-baseline > $o/nol2_$i.json 2> $o/nol2_$i.err || exit 1
done
for pf in 0.02 0.006 1.0; do
  MMRE_L1_PROBE_FRAC=$pf $T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu8_pf$pf.txt 2>&1 || exit 1
done
$T 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 --pack count > $o/emu8_count.txt 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_c2.log 2>&1 || exit 1
echo done
