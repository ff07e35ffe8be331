# Llama-3-8B (BASELINE config 2's model) with the round-5 kernels: aggregated bench at 64 and 256 in flight, ISL 5000.
set -o pipefail
mkdir -p gpurun_out
for c in 64 256; do
  timeout -k 10 400 python -u bench.py --model llama-3-8b --concurrency $c --steps 40 --warmup 10 > gpurun_out/r5ah_8b_c$c.log 2>&1
  rc=$?; echo "== c$c"; grep -E "timed step sizes" gpurun_out/r5ah_8b_c$c.log; grep -o '"value": [0-9.]*\|"p50_ttft_s": [0-9.]*' gpurun_out/r5ah_8b_c$c.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/r5ah_8b_c$c.log; exit $rc; }
done
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-8b --batch 64 --isl 5000 --steps 40 > gpurun_out/r5ah_8b_dec.log 2>&1
rc=$?; grep "decode batch" gpurun_out/r5ah_8b_dec.log; exit $rc
