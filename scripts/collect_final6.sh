#!/bin/bash
# Copy the judged artefacts of scripts/r6_final.sh from gpurun_out/final6 (scratch) into profiles/.
# usage: scripts/collect_final6.sh   (run in the build container after the parts came back)
cd "$(dirname "$0")/.."
f=gpurun_out/final6
mkdir -p profiles/r6
for j in $f/bench_*.json; do [ -s "$j" ] && cp "$j" profiles/r6/; done
for j in $f/ab_*.json; do [ -s "$j" ] && cp "$j" profiles/r6/ab/; done
for d in $f/prof_*/; do
  n=$(basename "$d"); n=${n#prof_}
  s=$(ls "$d"/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$s" ] && cp "$s" profiles/r6/${n}_kernel_stats.csv
done
[ -f $f/pytest_gpu.log ] && cp $f/pytest_gpu.log profiles/r6/pytest_gpu_final.log
for c in c1 c2 c2_tc c3 c4 c5 ns ns_distmult ns_complex ns_rotate; do
  [ -d gpurun_out/pmc_final6_$c ] && python scripts/pmc_summary.py final6_$c --json profiles/pmc_$c.json > /dev/null
done
ls -la profiles/r6 profiles/pmc_*.json
[ -f gpurun_out/final6/smoke.log ] && grep -v amdgpu gpurun_out/final6/smoke.log > profiles/r6/smoke_final.log
[ -f gpurun_out/final6/emu8.txt ] && (for w in 2 4 8; do grep -v amdgpu gpurun_out/final6/emu$w.txt; done) > profiles/r6/c2_shard_emulation.txt
[ -f gpurun_out/final6/emu8_c4.txt ] && grep -v amdgpu gpurun_out/final6/emu8_c4.txt > profiles/r6/c4_shard_emulation.txt
[ -f gpurun_out/final6/emu8_c5_entity.txt ] && grep -v amdgpu gpurun_out/final6/emu8_c5_entity.txt > profiles/r6/c5_entity_shard_emulation.txt
