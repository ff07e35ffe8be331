# Decode step with the batch held full through the timed window (bench_decode.py sizes
# max_tokens past the prefill phase): TP1 70B at 64, one TP2-shard rank at 64/96/128.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/dtp2.log
: > $L
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --batch 64 --steps 30 >> $L 2>&1 || { echo "tp1 failed"; tail -20 $L; exit 1; }
for b in 64 96 128; do
  timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --tp-shard 2 --batch $b --steps 30 >> $L 2>&1 || { echo "shard $b failed"; tail -20 $L; exit 1; }
done
grep "ms/step\|WARN" $L
