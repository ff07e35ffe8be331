# fp8 grouped GEMM at two workgroups per CU: numerics, microbenchmark, gpt-oss-120b fp8 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "moe or fp8" > gpurun_out/moe_occ_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/moe_occ_tests.log; exit 1; }
tail -1 gpurun_out/moe_occ_tests.log
timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_occ_bench.log 2>&1 || { echo "bench_moe failed"; tail -20 gpurun_out/moe_occ_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/moe_occ_bench.log
timeout -k 10 400 python bench.py --model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10 --quantization fp8 --concurrency 128 > gpurun_out/gptoss_fp8_c128_occ.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/gptoss_fp8_c128_occ.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gptoss_fp8_c128_occ.log | cut -c1-330
