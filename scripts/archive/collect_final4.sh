#!/bin/bash
# Copy the judged artefacts of scripts/r4_final.sh from gpurun_out/final4 (scratch) into profiles/.
# usage: scripts/collect_final4.sh   (run in the build container after the parts came back)
cd "$(dirname "$0")/../.."
f=gpurun_out/final4
mkdir -p profiles/r4
for j in $f/bench_*.json; do [ -s "$j" ] && cp "$j" profiles/r4/; done
for d in $f/prof_*/; do
  n=$(basename "$d"); n=${n#prof_}
  s=$(ls "$d"/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$s" ] && cp "$s" profiles/r4/${n}_kernel_stats.csv
done
[ -f $f/pytest_gpu.log ] && cp $f/pytest_gpu.log profiles/r4/pytest_gpu_final.log
for c in c1 c2 c3 c4 c5 ns ns_distmult ns_complex ns_rotate; do
  [ -d gpurun_out/pmc_final4_$c ] && python scripts/pmc_summary.py final4_$c --json profiles/pmc_$c.json > /dev/null
done
ls -la profiles/r4 profiles/pmc_*.json
