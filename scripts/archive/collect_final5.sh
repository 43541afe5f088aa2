#!/bin/bash
# Copy the judged artefacts of scripts/r5_final.sh from gpurun_out/final5 (scratch) into profiles/.
# usage: scripts/collect_final5.sh   (run in the build container after the parts came back)
cd "$(dirname "$0")/../.."
f=gpurun_out/final5
mkdir -p profiles/r5
for j in $f/bench_*.json; do [ -s "$j" ] && cp "$j" profiles/r5/; done
for j in $f/ab_*.json; do [ -s "$j" ] && cp "$j" profiles/r5/ab/; done
for d in $f/prof_*/; do
  n=$(basename "$d"); n=${n#prof_}
  s=$(ls "$d"/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$s" ] && cp "$s" profiles/r5/${n}_kernel_stats.csv
done
[ -f $f/pytest_gpu.log ] && cp $f/pytest_gpu.log profiles/r5/pytest_gpu_final.log
for c in c1 c2 c3 c4 c5 ns ns_distmult ns_complex ns_rotate; do
  [ -d gpurun_out/pmc_final5_$c ] && python scripts/pmc_summary.py final5_$c --json profiles/pmc_$c.json > /dev/null
done
ls -la profiles/r5 profiles/pmc_*.json
[ -f gpurun_out/final5/smoke.log ] && grep -v amdgpu gpurun_out/final5/smoke.log > profiles/r5/smoke_final.log
[ -f gpurun_out/final5/emu8.txt ] && (for w in 2 4 8; do grep -v amdgpu gpurun_out/final5/emu$w.txt; done) > profiles/r5/c2_shard_emulation.txt
