#!/bin/bash
# round 4, GPU call L: C2 A/B on one box -- this build vs the round-3 tree (ab_r3, a git worktree at db688e2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r4l
mkdir -p $o
T="timeout -k 10 300"
for i in 1 2; do
  $T python -u bench.py --steps 200 --no-cpu-baseline > $o/cur_$i.json 2> $o/cur_$i.err || exit 1
  (cd ab_r3 && $T python -u bench.py --steps 200 --no-cpu-baseline) > $o/r3_$i.json 2> $o/r3_$i.err || exit 1
  for v in v1 v2 v3; do
    MMRE_LIB=$PWD/ab/lib_$v.so $T python -u bench.py --steps 200 --no-cpu-baseline > $o/${v}_$i.json 2> $o/${v}_$i.err || exit 1
  done
done
$T python -u bench.py --config ns --steps 200 --no-cpu-baseline > $o/ns_cur.json 2> $o/ns_cur.err || exit 1
(cd ab_r3 && $T python -u bench.py --config ns --steps 200 --no-cpu-baseline) > $o/ns_r3.json 2> $o/ns_r3.err || exit 1
$T rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_cur -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_cur.log 2>&1 || exit 1
(cd ab_r3 && $T rocprofv3 --kernel-trace --stats --output-format csv -d ../$o/prof_r3 -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > ../$o/prof_r3.log 2>&1) || exit 1
MMRE_LIB=$PWD/ab/lib_v3.so timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_sweep_filters_gpu.py "tests/test_ref_fixture_gpu.py::test_reference_ranks_full_size[c2]" tests/test_link_gpu.py \
  > $o/pytest_v3.log 2>&1 || { echo "v3 pytest failed"; exit 1; }
echo done
