#!/bin/bash
# Kernel-trace averages of the NS step for library variants (in-tree "cur" and abl/abl_<name>.so),
# one rocprofv3 run each. usage: [BENCH_ARGS=...] scripts/trace_variants.sh <config> name1 [name2 ...]
cfg=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tv; rm -rf gpurun_out/tv/*
for v in cur "$@"; do
  if [ "$v" = cur ]; then L=; else L=abl/abl_$v.so; fi
  MMRE_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tv/$v -o run -- \
      python bench.py --config $cfg $BENCH_ARGS --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/tv/$v.log 2>&1 || exit $?
  echo "== $v"
  python - gpurun_out/tv/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if int(r["Calls"]) >= 20:
        print(f'{r["Name"][:70]:72s} {int(r["Calls"]):5d} {float(r["AverageNs"]) / 1e3:8.2f} us')
PY
done
