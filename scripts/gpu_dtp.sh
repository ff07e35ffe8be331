# Decode TP2 evidence on one GPU: (1) one rank of a TP2 Llama-3-70B decode
# replica (heads/FFN/vocab halved) at batch 64/96/128 vs the TP1 replica at 64;
# (2) 4-rank P/D rehearsal (2 prefill + one TP2 decode replica) on cuda:0.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/dtp.log
: > $L
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --batch 64 --steps 30 >> $L 2>&1 || { echo "tp1 failed"; tail -20 $L; exit 1; }
for b in 96 128; do
  timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --tp-shard 2 --batch $b --steps 30 >> $L 2>&1 || { echo "shard $b failed"; tail -20 $L; exit 1; }
done
grep "ms/step" $L
LLMD_BENCH_STACKS=200 LLMD_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --mode pd --prefill-gpus 2 \
  --steps 30 --warmup 5 --model llama-3-8b --kv-cache-gb 8 --concurrency 8 > gpurun_out/pd_dtp_rehearsal.log 2>&1 || { echo "pd dtp failed"; tail -40 gpurun_out/pd_dtp_rehearsal.log; exit 1; }
grep '^{' gpurun_out/pd_dtp_rehearsal.log | cut -c1-600
