#!/bin/bash
# Round 6, call l: the fused L1 evaluation with the filter counts after the sweeps (K3 split) and
# a deeper probe loop -- tests, then N = 1 and 8-way A/B (MMRE_EVAL_SPLIT_K3=0 / 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6l
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_eval_fused_gpu.py tests/test_sweep_filters_gpu.py tests/test_sharding_gloo.py tests/test_ref_fixture_gpu.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for v in 1 0; do
  MMRE_EVAL_SPLIT_K3=$v timeout -k 10 300 python -u scripts/step_breakdown.py --emulate-world 8 --graph --config c2 > $o/emu_s$v.txt 2>&1 || { tail -20 $o/emu_s$v.txt; exit 1; }
  grep -E "^N=1|^rank|^c2 world" $o/emu_s$v.txt | sed "s/^/split$v: /" | cut -c1-120
done
MMRE_EVAL_SPLIT_K3=1 timeout -k 10 400 python bench.py --no-cpu-baseline > $o/c2_s1.json 2> $o/c2_s1.err || exit 1
MMRE_EVAL_SPLIT_K3=0 timeout -k 10 400 python bench.py --no-cpu-baseline > $o/c2_s0.json 2> $o/c2_s0.err || exit 1
python -c "import json; [print(t, json.load(open('$o/c2_'+t+'.json'))['ms_per_step']) for t in ('s1','s0')]"
echo done
