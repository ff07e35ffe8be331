# P/D rehearsal of the 8-GPU topology on one GPU: 8 ranks (6 prefill + 2 decode) on cuda:0, small model.
set -o pipefail
mkdir -p gpurun_out
LLMD_BENCH_STACKS=200 LLMD_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 30 --warmup 5 \
  --model llama-3-8b --kv-cache-gb 8 --concurrency 16 > gpurun_out/pd8_rehearsal.log 2>&1 || { echo "pd8 failed"; tail -40 gpurun_out/pd8_rehearsal.log; exit 1; }
grep '^{' gpurun_out/pd8_rehearsal.log | cut -c1-400
