# fp8 MoE v3 with the fused activation quantisation: numerics, microbenchmark, gpt-oss-120b fp8 end to end
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_kv.py -x -q --timeout 120 --timeout-method thread -k "moe" > gpurun_out/moe_fq_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/moe_fq_tests.log; exit 1; }
tail -1 gpurun_out/moe_fq_tests.log
timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_fq_bench.txt 2>&1 || { echo bench failed; tail -20 gpurun_out/moe_fq_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/moe_fq_bench.txt | grep "T=4096\|T=5120"
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10 --quantization fp8"
for c in 128 256; do
  timeout -k 10 400 python bench.py $M --concurrency $c > gpurun_out/gptoss_fq_c$c.log 2>&1 || { echo "c$c failed"; tail -20 gpurun_out/gptoss_fq_c$c.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/gptoss_fq_c$c.log | grep "timed\|^{" | cut -c1-200
done
