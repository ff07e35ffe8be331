#!/bin/bash
# GPU validation chain used with gpurun: unit tests, smoke, P/D rehearsal, 70B bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || exit $?
echo "gpu tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
echo "smoke ok"
if [ -n "$PD4" ]; then
LLMD_BENCH_STACKS=200 LLMD_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 30 --warmup 5 \
  --model llama-3-8b --kv-cache-gb 12 --concurrency 16 > gpurun_out/pd4_rehearsal.log 2>&1 || exit $?
echo "pd4 ok"
fi
if [ -n "$BENCH70" ]; then
timeout -k 10 900 python bench.py --json-out gpurun_out/bench70.json > gpurun_out/bench70.log 2>&1 || exit $?
echo "bench70 ok"
fi
