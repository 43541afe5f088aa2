mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_m3ae_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m3ae_tests.log 2>&1; rc=$?
tail -2 gpurun_out/m3ae_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --config m3ae --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_m3ae.log 2>&1 || exit 1
tail -1 gpurun_out/bench_m3ae.log | cut -c1-700
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_m3ae_$1 -o run -- python bench.py --config m3ae --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_m3ae_$1.log 2>&1
echo prof rc=$?
