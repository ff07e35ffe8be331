# MoE glue trimmed (no arange/where/fill per MoE call): numerics over every MoE path, microbench, gpt-oss bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_kv.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_deepseek.py tests/test_ep_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/moe_glue_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/moe_glue_tests.log; exit 1; }
tail -1 gpurun_out/moe_glue_tests.log
timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_glue_bench.log 2>&1 || { echo "bench_moe failed"; tail -20 gpurun_out/moe_glue_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/moe_glue_bench.log
timeout -k 10 400 python bench.py --model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10 --quantization fp8 --concurrency 128 > gpurun_out/gptoss_fp8_c128_glue.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/gptoss_fp8_c128_glue.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gptoss_fp8_c128_glue.log | cut -c1-330
