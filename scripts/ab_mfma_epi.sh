#!/bin/bash
# A/B of the MFMA sweep's stage size (MMRE_MFMA_STAGE 32: 2 workgroups / CU, register row
# counters; 16: 4 workgroups / CU, ballot row counters) and grid (MMRE_SWEEP_GRID) at C3 / C5:
# sweep kernel ms from the bench's events.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "c3 100" "c5 15"; do
  set -- $cfg
  for spec in "32 " "16 " "16 1024" "16 3072" "16 4096"; do
    set -- $1 $2 $spec
    tag=$1_$3_${4:-auto}
    MMRE_MFMA_STAGE=$3 MMRE_SWEEP_GRID=$4 timeout -k 10 240 python bench.py --config $1 --steps $2 --warmup 3 \
        --no-cpu-baseline > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; exit 1; }
    echo "$tag $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_$tag.log) $(grep -o '"frac": [0-9.]*' gpurun_out/ab_$tag.log)"
  done
done
