# fp8 grouped GEMM: MFMA E8M0 hardware scales vs VALU block re-scaling (A/B), plus the fp8 GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_kv.py tests/test_deepseek.py -x -q --timeout 120 --timeout-method thread > gpurun_out/moe_hws_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/moe_hws_tests.log; exit 1; }
tail -1 gpurun_out/moe_hws_tests.log
timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_hws_bench.txt 2>&1 || { echo bench failed; tail -20 gpurun_out/moe_hws_bench.txt; exit 1; }
LLMD_MOE_FP8_SOFT_SCALE=1 timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_soft_bench.txt 2>&1 || { echo bench failed; exit 1; }
echo "== hardware E8M0 scales"; grep -v amdgpu.ids gpurun_out/moe_hws_bench.txt
echo "== VALU block re-scaling"; grep -v amdgpu.ids gpurun_out/moe_soft_bench.txt
