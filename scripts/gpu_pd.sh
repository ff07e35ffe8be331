# P/D rehearsal on one GPU: 4 ranks (3 prefill + 1 decode) on cuda:0 with a small model, gloo control.
set -o pipefail
mkdir -p gpurun_out
LLMD_BENCH_STACKS=200 LLMD_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --mode pd --steps 30 --warmup 5 \
  --model llama-3-8b --kv-cache-gb 12 --concurrency 16 > gpurun_out/pd4_rehearsal.log 2>&1 || { echo "pd4 failed"; tail -40 gpurun_out/pd4_rehearsal.log; exit 1; }
grep '^{' gpurun_out/pd4_rehearsal.log
