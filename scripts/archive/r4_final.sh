#!/bin/bash
# Round-4 final measurements on the GPU box, in parts (each fits one gpurun call):
#   A: full -m gpu suite + smoke + C2 bench line + C2 kernel trace
#   B: C1 / C3 / C4 / C5 bench lines (cpu_baseline + reference parity legs) + kernel traces
#   C: NS bench lines (TransE k 25 / k 10 with the reference CPU leg; DistMult / ComplEx / RotatE) + traces
#   D1 / D2: PMC passes (scripts/pmc.sh) of c1 c2 c4 ns / c3 c5; E: C1 PMC + C2 bench again; F: C1 bench again;
#   G: PMC passes of the DistMult / ComplEx / RotatE NS steps; H: their bench lines again
# usage: scripts/r4_final.sh <A|B|C|D1|D2|E|F|G|H>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/final4
mkdir -p $o
trace() {  # <name> <bench args...>
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$n -o run -- \
    python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline > $o/prof_$n.log 2>&1
}
case $1 in
  A)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || exit $?
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
    timeout -k 10 300 python bench.py > $o/bench_c2.json 2> $o/bench_c2.err || exit $?
    trace c2 --config c2 || exit $?
    ;;
  B)
    for c in c1 c3 c4 c5; do
      timeout -k 10 400 python bench.py --config $c > $o/bench_$c.json 2> $o/bench_$c.err || exit $?
      trace $c --config $c || exit $?
    done
    ;;
  C)
    timeout -k 10 300 python bench.py --config ns > $o/bench_ns.json 2> $o/bench_ns.err || exit $?
    timeout -k 10 300 python bench.py --config ns --ns-neg 10 > $o/bench_ns_k10.json 2> $o/bench_ns_k10.err || exit $?
    trace ns --config ns || exit $?
    for m in distmult complex rotate; do
      timeout -k 10 300 python bench.py --config ns --ns-model $m --no-cpu-baseline > $o/bench_ns_$m.json 2> $o/bench_ns_$m.err || exit $?
      trace ns_$m --config ns --ns-model $m || exit $?
    done
    ;;
  D1)
    for c in c1 c2 c4 ns; do bash scripts/pmc.sh final4_$c --config $c || exit $?; done
    ;;
  D2)
    for c in c3 c5; do bash scripts/pmc.sh final4_$c --config $c || exit $?; done
    ;;
  E)  # C1's PMC passes, then the C2 bench line again (its PMC summary installed in profiles/ by now)
    bash scripts/pmc.sh final4_c1 --config c1 || exit $?
    timeout -k 10 300 python bench.py > $o/bench_c2.json 2> $o/bench_c2.err || exit $?
    ;;
  G)  # PMC passes of the other models' NS steps (profiles/pmc_ns_<model>.json)
    for m in distmult complex rotate; do bash scripts/pmc.sh final4_ns_$m --config ns --ns-model $m || exit $?; done
    ;;
  H)  # the other models' NS lines again, with their PMC summaries installed
    for m in distmult complex rotate; do
      timeout -k 10 300 python bench.py --config ns --ns-model $m --no-cpu-baseline > $o/bench_ns_$m.json 2> $o/bench_ns_$m.err || exit $?
    done
    ;;
  F)  # the C1 bench line with its PMC summary installed
    timeout -k 10 300 python bench.py --config c1 > $o/bench_c1.json 2> $o/bench_c1.err || exit $?
    ;;
esac
