#!/bin/bash
# Round-3 full GPU check: the -m gpu suite, then N = 2 / 8 bench rehearsals (gloo, every rank
# on cuda:0) of the relation- and entity-sharded paths with the per-rank breakdown.
set -o pipefail
tag=${1:-full}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r3_gpu_$tag.log 2>&1 || exit $?
fi
for n in 2 8; do
  MMRE_BENCH_GLOO=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/r3_rehearsal_n${n}_$tag.json 2> gpurun_out/r3_rehearsal_n${n}_$tag.err || exit $?
done
MMRE_BENCH_GLOO=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 8 --steps 10 --warmup 2 --no-cpu-baseline \
  --config c5 --shard entity > gpurun_out/r3_rehearsal_n8_c5_entity_$tag.json 2> gpurun_out/r3_rehearsal_n8_c5_entity_$tag.err
