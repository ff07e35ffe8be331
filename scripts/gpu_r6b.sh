# Round 6: fp8 prefill GEMM numerics + microbench (then the steady-state benches).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_pgemm_fp8.py tests/test_collective_failure.py > gpurun_out/r6b_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r6b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_pgemm_fp8.py > gpurun_out/r6b_pgemm8.log 2>&1
rc=$?; cat gpurun_out/r6b_pgemm8.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6a.sh
