#!/bin/bash
# Hardware-counter passes for the bench workload (one counter group per rocprofv3 run, no
# tracing domains combined with --pmc). usage: scripts/pmc.sh <tag> [bench args...]
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
# the binary these counters belong to (bench.py reports traffic only for this build)
python -c "import hashlib; print(hashlib.sha256(open('multimodal-relation-extrapolation_amd/mmre/lib/libmmre_hip.so','rb').read()).hexdigest()[:16])" > $out/lib_sha256.txt
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $out/p$i.log; exit $rc; fi
done
