#!/bin/bash
# round 4: 8-bit SAD probes -- v_sad_u8 issue rate and the undecided fraction of an 8-bit L1 code filter at C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/probe8
mkdir -p $o
timeout -k 10 120 ./scripts/probes/sad8_rate > $o/sad8_rate.txt 2>&1 || exit 1
timeout -k 10 400 python -u scripts/probes/transe_quant_frac.py > $o/quant_frac.txt 2>&1 || exit 1
echo done
