# fp8 W8A8 + fp8 KV Llama-3-70B after the scaled-GEMM TunableOp entries: decode step and the serving bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --batch 64 --isl 5000 --steps 30 2>&1 | grep "ms/step" | sed 's/^/after: /' || exit 1
timeout -k 10 600 python -u bench.py --quantization fp8 --kv-cache-dtype fp8 --steps 40 --warmup 20 > gpurun_out/bench_fp8_after.log 2>&1 || { tail -20 gpurun_out/bench_fp8_after.log; exit 1; }
grep "timed step\|^{" gpurun_out/bench_fp8_after.log | cut -c1-330
