#!/bin/bash
# Round 6, call r: C5 A/B of the wide sweep's decision-pass variants (scripts/variants.txt) on one
# box: previous build, thresholds only, + screen, + C = 0 first stage, all three (in-tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6r
mkdir -p $o
T="timeout -k 10"
for rep in 1 2; do
for v in head_82df655 w_thr w_screen w_zeroc shipped; do
  if [ $v = shipped ]; then L=multimodal-relation-extrapolation_amd/mmre/lib/libmmre_hip.so; else L=abl/$v.so; fi
  MMRE_LIB=$L $T 400 python -u bench.py --config c5 --no-cpu-baseline --steps 30 --warmup 3 > $o/c5_${v}_$rep.json 2> $o/c5_${v}_$rep.err || { tail -20 $o/c5_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$o/c5_${v}_$rep.json'));r=d['roofline'];print('c5 $v',round(d['ms_per_step'],4),round(r['kernel_ms'],4),round(r['frac'],3),d['mfma_filter']['undecided_pairs'])"
done
done
echo done
