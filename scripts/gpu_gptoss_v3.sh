# gpt-oss-120b fp8 on one MI355X after the 256-row fp8 grouped GEMM: 128 and 256 in flight, ISL 5150 / OSL 250
set -o pipefail
mkdir -p gpurun_out
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10 --quantization fp8"
for c in 128 256; do
  timeout -k 10 400 python bench.py $M --concurrency $c > gpurun_out/gptoss_v3_c$c.log 2>&1 || { echo "c$c failed"; tail -20 gpurun_out/gptoss_v3_c$c.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/gptoss_v3_c$c.log | cut -c1-330
done
