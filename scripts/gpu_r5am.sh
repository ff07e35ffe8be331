# Rehearsal of the driver's multi-GPU bench topologies on ONE GPU (all ranks on cuda:0, gloo control,
# small model): N=2 aggregated (dp2) and N=8 P/D (6 prefill + one TP2 decode replica).
set -o pipefail
mkdir -p gpurun_out
export LLMD_BENCH_DEVICE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29523 bench.py --gpus 2 --steps 20 --warmup 5 --model llama-3-8b --kv-cache-gb 16 --concurrency 16 \
  > gpurun_out/agg2_rehearsal_r5b.log 2>&1 || { echo "agg2 failed"; tail -40 gpurun_out/agg2_rehearsal_r5b.log; exit 1; }
grep '^{' gpurun_out/agg2_rehearsal_r5b.log | cut -c1-300
LLMD_BENCH_STACKS=200 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 30 --warmup 5 --model llama-3-8b \
  --kv-cache-gb 8 --concurrency 16 > gpurun_out/pd8_rehearsal_r5b.log 2>&1 || { echo "pd8 failed"; tail -40 gpurun_out/pd8_rehearsal_r5b.log; exit 1; }
grep '^{' gpurun_out/pd8_rehearsal_r5b.log | cut -c1-400
