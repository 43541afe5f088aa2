#!/bin/bash
# Round 5, GPU call L (session 2: the tree was restored from HEAD 10b1caf, earlier results lost):
# the full -m gpu suite + smoke on the current build, C2 lines (two streams = bench default, and
# one), a C2 kernel trace, the relation-sharded emulation at 2 / 4 / 8 ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5l
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
$T 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
$T 600 python -u bench.py > $o/c2.json 2> $o/c2.err || { tail -20 $o/c2.err; exit 1; }
$T 300 python -u bench.py --steps 200 --no-cpu-baseline --eval-streams 1 > $o/c2_s1.json 2> $o/c2_s1.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_c2.log 2>&1 || exit 1
for w in 2 4 8; do
  $T 300 python -u scripts/step_breakdown.py --emulate-world $w --graph --config c2 > $o/emu$w.txt 2>&1 || exit 1
done
echo done
