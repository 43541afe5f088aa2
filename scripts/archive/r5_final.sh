#!/bin/bash
# Round-5 final measurements on the GPU box, in parts (each fits one gpurun call):
#   T: full -m gpu suite + smoke + the 2 / 4 / 8-way C2 emulation
#   P1 / P2: PMC passes (scripts/pmc.sh) of c1 c2 c4 ns / c3 c5 ns_distmult ns_complex ns_rotate
#   B1: C1 / C2 / C3 lines (cpu_baseline + reference parity legs) + kernel traces
#   B2: C4 / C5 lines + traces;  B3: NS lines (TransE k 25 / k 10, DistMult, ComplEx, RotatE) + traces
# usage: scripts/r5_final.sh <T|P1|P2|B1|B2|B3>
set -o pipefail
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
  T)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
    tail -2 $o/pytest_gpu.log
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || exit 1
    for w in 2 4 8; do
      timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world $w --graph --config c2 > $o/emu$w.txt 2>&1 || exit 1
    done
    ;;
  P1)
    for c in c1 c2 c4; do bash scripts/pmc.sh final5_$c --config $c || exit 1; done
    bash scripts/pmc.sh final5_ns --config ns || exit 1
    ;;
  P2)
    for c in c3 c5; do bash scripts/pmc.sh final5_$c --config $c || exit 1; done
    for m in distmult complex rotate; do bash scripts/pmc.sh final5_ns_$m --config ns --ns-model $m || exit 1; done
    ;;
  B1)
    for c in c1 c2 c3; do
      timeout -k 10 400 python bench.py --config $c > $o/bench_$c.json 2> $o/bench_$c.err || exit 1
      trace $c --config $c || exit 1
    done
    ;;
  B2)
    for c in c4 c5; do
      timeout -k 10 500 python bench.py --config $c > $o/bench_$c.json 2> $o/bench_$c.err || exit 1
      trace $c --config $c || exit 1
    done
    # A/B on the same box: C5 on the 128 x 128 split-bf16 sweep
    MMRE_BF3_WIDE=0 timeout -k 10 500 python bench.py --config c5 --no-cpu-baseline > $o/ab_c5_narrow.json 2> $o/ab_c5_narrow.err || exit 1
    ;;
  B3)
    timeout -k 10 300 python bench.py --config ns > $o/bench_ns.json 2> $o/bench_ns.err || exit 1
    timeout -k 10 300 python bench.py --config ns --ns-neg 10 > $o/bench_ns_k10.json 2> $o/bench_ns_k10.err || exit 1
    trace ns --config ns || exit 1
    for m in distmult complex rotate; do
      timeout -k 10 300 python bench.py --config ns --ns-model $m --no-cpu-baseline > $o/bench_ns_$m.json 2> $o/bench_ns_$m.err || exit 1
      trace ns_$m --config ns --ns-model $m || exit 1
    done
    ;;
esac
echo "part $1 done"
