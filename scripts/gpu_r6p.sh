# bf16 persistent MoE numerics + v4/v8 timing, then gpt-oss fp8 serving v4 vs v8 (steady-state window)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bf16_v4" > gpurun_out/r6p_test.log 2>&1 || { tail -40 gpurun_out/r6p_test.log; exit 1; }
tail -2 gpurun_out/r6p_test.log
timeout -k 10 400 python -u scripts/bench_moe8.py > gpurun_out/r6p_bench.log 2>&1 || { cat gpurun_out/r6p_bench.log; exit 1; }
cat gpurun_out/r6p_bench.log
bash scripts/gpu_r6o.sh
