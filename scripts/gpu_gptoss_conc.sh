# gpt-oss-120b on one MI355X: concurrency sweep (fp8 experts, then bf16) at ISL 5150 / OSL 250.
set -o pipefail
mkdir -p gpurun_out
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10"
for c in 256; do
  timeout -k 10 400 python bench.py $M --quantization fp8 --concurrency $c > gpurun_out/gptoss_fp8_c$c.log 2>&1 || { echo "fp8 c$c failed"; tail -20 gpurun_out/gptoss_fp8_c$c.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/gptoss_fp8_c$c.log | cut -c1-330
  grep -o '"p50_ttft_s": [0-9.]*' gpurun_out/gptoss_fp8_c$c.log
done
timeout -k 10 400 python bench.py $M --concurrency 112 > gpurun_out/gptoss_bf16_c112.log 2>&1 || { echo "bf16 failed"; tail -20 gpurun_out/gptoss_bf16_c112.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gptoss_bf16_c112.log | cut -c1-330
