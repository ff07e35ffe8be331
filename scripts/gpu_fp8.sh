set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fp8_kv.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fp8_tests.log; exit 1; }
tail -2 gpurun_out/fp8_tests.log
timeout -k 10 200 python scripts/bench_attn.py > gpurun_out/attn_bf16.txt 2>&1 && timeout -k 10 200 python scripts/bench_attn.py --kv-dtype fp8 > gpurun_out/attn_fp8.txt 2>&1 && cat gpurun_out/attn_bf16.txt gpurun_out/attn_fp8.txt
