#!/bin/bash
# NS training step for every model at the C2 training shape: bench line + kernel trace each.
# usage: scripts/ns_models.sh <tag> [models...]
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${@:-distmult complex rotate}; do
  timeout -k 10 240 python bench.py --config ns --ns-model $m --no-cpu-baseline > gpurun_out/ns_${m}_$tag.json 2> gpurun_out/ns_${m}_$tag.err || exit $?
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns_${m}_$tag -o run -- \
      python bench.py --config ns --ns-model $m --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/prof_ns_${m}_$tag.log 2>&1 || exit $?
  echo "== $m $(python -c "import json,sys; d=json.loads(open('gpurun_out/ns_${m}_$tag.json').read().strip().splitlines()[-1]); print('step_ms %.4f fused_ms %.4f' % (d['ms_per_step'], d['roofline']['kernel_ms']))")"
  python - gpurun_out/prof_ns_${m}_$tag <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if int(r["Calls"]) >= 20:
        print(f'   {r["Name"][:70]:72s} {int(r["Calls"]):5d} {float(r["AverageNs"]) / 1e3:8.2f} us')
PY
done
