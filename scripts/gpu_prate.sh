# Prefill-only rate of one 70B P/D prefill rank (ISL 5000, max_tokens=1, chunks of 8192) and
# the TP2-shard decode step at batch 80 / 112 (see scripts/gpu_dtp.sh).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/prate.log
: > $L
timeout -k 10 400 python -u scripts/bench_prefill_rate.py --steps 12 >> $L 2>&1 || { echo "prefill rate failed"; tail -20 $L; exit 1; }
for b in 80 112; do
  timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --tp-shard 2 --batch $b --steps 30 >> $L 2>&1 || { echo "shard $b failed"; tail -20 $L; exit 1; }
done
grep "ms/step\|tok/s" $L
