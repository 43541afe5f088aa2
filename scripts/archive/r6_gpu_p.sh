#!/bin/bash
# Round 6, call p: stall attribution of the wide split-bf16 sweep at C5 -- ablation libraries
# (scripts/variants.txt): decision pass out (w_noepi), + half the LDS operand reads (w_halflds),
# + no entity-row DMA (w_noedma), + no DMA of either operand (w_nodma). Timing only: the
# ablations' counts are wrong by construction.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6p
mkdir -p $o
T="timeout -k 10"
for v in shipped w_noepi w_halflds w_noedma w_nodma shipped w_noepi; do
  if [ $v = shipped ]; then L=multimodal-relation-extrapolation_amd/mmre/lib/libmmre_hip.so; else L=abl/$v.so; fi
  MMRE_LIB=$L $T 400 python -u bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $o/c5_$v.json 2> $o/c5_$v.err || { tail -20 $o/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/c5_$v.json'));r=d['roofline'];print('c5 $v',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(r['frac'],3))"
done
echo done
