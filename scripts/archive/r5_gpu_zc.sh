#!/bin/bash
# Round 5, GPU call ZC: the in-tree build with the wide split-bf16 sweep as the C5 default:
# the MFMA-filter tests (128 x 128 and wide at QT 256 / 128), the C3 / C5 reference fixtures,
# smoke, and the C5 / C3 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/r5zc
mkdir -p $o
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sweep_filters_gpu.py tests/test_link_gpu.py \
  > $o/pytest_filters.log 2>&1 || { tail -40 $o/pytest_filters.log; exit 1; }
tail -1 $o/pytest_filters.log
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_ref_fixture_gpu.py \
  > $o/pytest_fix.log 2>&1 || { tail -40 $o/pytest_fix.log; exit 1; }
tail -1 $o/pytest_fix.log
$T 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || exit 1
for c in c5 c3; do
  $T 400 python -u bench.py --config $c > $o/bench_$c.json 2> $o/bench_$c.err || exit 1
  python -c "import json;d=json.load(open('$o/bench_$c.json'));r=d['roofline'];print('$c',round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3), d.get('parity',{}).get('mismatches') if isinstance(d.get('parity'),dict) else '')"
done
MMRE_BF3_WIDE=1 $T 400 python -u bench.py --config c3 --no-cpu-baseline > $o/bench_c3_wide.json 2> $o/bench_c3_wide.err || exit 1
python -c "import json;d=json.load(open('$o/bench_c3_wide.json'));r=d['roofline'];print('c3 wide',round(d['ms_per_step'],4),r['kernel'],round(r['kernel_ms'],4),round(r['frac'],3))"
echo done
