# MoE grouped GEMMs: numerics (bf16 + block-fp8), then the bf16 vs fp8 microbenchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_kv.py tests/test_deepseek.py -x -q --timeout 120 --timeout-method thread -k "moe or deepseek" -m gpu > gpurun_out/moe_tests.log 2>&1 || { echo "moe tests failed"; tail -40 gpurun_out/moe_tests.log; exit 1; }
tail -1 gpurun_out/moe_tests.log
timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/moe_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/moe_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/moe_bench.log
