#!/bin/bash
# Round 5, GPU call ZA: where the C5 split-bf16 sweep's time goes. (1) the wide sweep with its
# decision pass compiled out (abl/bf3w_noepi.so: counts wrong, timing only) against the full
# one; (2) stall / issue counters of the wide and the 128 x 128 sweeps (abl/bf3w.so,
# MMRE_BF3_WIDE=1 / 0), one counter group per rocprofv3 run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5za
mkdir -p $o
T="timeout -k 10"
for v in bf3w_noepi bf3w; do
  MMRE_LIB=abl/$v.so $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_$v -o run -- \
    python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --eval-streams 1 > $o/tr_$v.log 2>&1 || exit 1
  grep "k_sweep_bf3" $o/tr_$v/run_kernel_stats.csv | awk -F'",' '{print "'$v'", $2}'
done
i=0
for w in 1 0; do
  for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
             "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    MMRE_LIB=abl/bf3w.so MMRE_BF3_WIDE=$w timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $o/w${w}_p$i -o run -- \
      python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --eval-streams 1 > $o/w${w}_p$i.log 2>&1
    rc=$?
    echo "wide=$w pass $i ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $o/w${w}_p$i.log; exit $rc; fi
  done
done
echo done
