# round 4 (v): gpt-oss-120b (the reference's published P/D model) on one MI355X with the round-4 kernels
# (MoE v3 bf16/fp8 schedules, hybrid sliding-window KV) at ISL 5150 / OSL 250
set -o pipefail
mkdir -p gpurun_out
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10"
for c in 128 256; do
  timeout -k 10 500 python bench.py $M --quantization fp8 --concurrency $c > gpurun_out/r4v_fp8_c$c.out 2> gpurun_out/r4v_fp8_c$c.err || { echo "fp8 c$c failed"; tail -20 gpurun_out/r4v_fp8_c$c.err; exit 1; }
  grep "timed step" gpurun_out/r4v_fp8_c$c.err | tail -1
  tail -1 gpurun_out/r4v_fp8_c$c.out | cut -c1-200; grep -o '"p50_ttft_s": [0-9.]*' gpurun_out/r4v_fp8_c$c.out
done
for c in 64 112; do
  timeout -k 10 500 python bench.py $M --concurrency $c > gpurun_out/r4v_bf16_c$c.out 2> gpurun_out/r4v_bf16_c$c.err || { echo "bf16 c$c failed"; tail -20 gpurun_out/r4v_bf16_c$c.err; exit 1; }
  grep "timed step" gpurun_out/r4v_bf16_c$c.err | tail -1
  tail -1 gpurun_out/r4v_bf16_c$c.out | cut -c1-200; grep -o '"p50_ttft_s": [0-9.]*' gpurun_out/r4v_bf16_c$c.out
done
