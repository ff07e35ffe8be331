# Round 6: persistent fp8 prefill GEMM - numerics, then the 70B-shape A/B against the tiled form and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pgemm_fp8.py > gpurun_out/r6g_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r6g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_pgemm_fp8.py --m 4608,5063,8192 > gpurun_out/r6g_pgemm8.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6g_pgemm8.log; exit $rc
