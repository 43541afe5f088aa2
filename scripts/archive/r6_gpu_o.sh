#!/bin/bash
# Round 6, call o: the split-bf16 sweep's whole-round grid -- filter parity tests, C3 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r6o
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
for t in a g768 b; do
  if [ $t = g768 ]; then export MMRE_SWEEP_GRID=768; else unset MMRE_SWEEP_GRID; fi
  timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 50 --warmup 5 > $o/c3_$t.json 2> $o/c3_$t.err || { tail -20 $o/c3_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c3_$t.json')); print('c3 $t', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3), d['parity'].get('mismatches') if isinstance(d.get('parity'),dict) else None)"
done
echo done
