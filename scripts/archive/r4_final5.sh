#!/bin/bash
# Round 4, final build (tight L1 bound): the parts that depend on the TransE L1 sweep.
#   X: PMC passes of C2 / C1 (summaries written into profiles/ on the box and copied to
#      gpurun_out/final5), full -m gpu suite, smoke, C2 bench line + kernel trace
#   Y: C1 bench line + trace, per-rank C2 shard emulations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/final5
mkdir -p $o
trace() {  # <name> <bench args...>
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$n -o run -- \
    python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_$n.log 2>&1
}
case $1 in
  X)
    for c in c2 c1; do
      bash scripts/pmc.sh final5_$c --config $c || exit $?
      python scripts/pmc_summary.py final5_$c --json profiles/pmc_$c.json > /dev/null || exit 1
      cp profiles/pmc_$c.json $o/pmc_$c.json
    done
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || exit $?
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
    timeout -k 10 300 python bench.py > $o/bench_c2.json 2> $o/bench_c2.err || exit $?
    trace c2 --config c2 || exit $?
    ;;
  Y)
    timeout -k 10 400 python bench.py --config c1 > $o/bench_c1.json 2> $o/bench_c1.err || exit $?
    trace c1 --config c1 || exit $?
    rm -f $o/c2_shard_emulation.txt
    for W in 2 4 8; do
      timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world $W --graph --config c2 >> $o/c2_shard_emulation.txt 2>&1 || exit 1
    done
    timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world 8 --entity --config c2 >> $o/c2_shard_emulation.txt 2>&1 || exit 1
    ;;
esac
