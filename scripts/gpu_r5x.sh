# Padding slots / W rows past N / A rows past M read out-of-range zeros instead of a clamped real row:
# numerics of every affected kernel first, then the MoE A/B and the power probe's MoE arms.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_fp8_kv.py tests/test_mgemm.py -k "moe or pgemm" > gpurun_out/r5x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5x_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_moe.py > gpurun_out/r5x_moe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5x_moe.log | grep -E "T=4096|T=5120"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/gemm_clock_probe.py moe > gpurun_out/r5x_clock.log 2>&1
rc=$?; grep "TF/s" gpurun_out/r5x_clock.log; exit $rc
