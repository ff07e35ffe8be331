set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "mgemm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mgemm_fp8_test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/mgemm_fp8_test.log; exit 1; }
tail -1 gpurun_out/mgemm_fp8_test.log
timeout -k 10 600 python -u scripts/sweep_mgemm_fp8.py --model llama-3-70b > gpurun_out/mgemm_fp8_sweep_70b.log 2>&1 || { echo "sweep failed"; tail -30 gpurun_out/mgemm_fp8_sweep_70b.log; exit 1; }
grep -v "^ROW\|amdgpu" gpurun_out/mgemm_fp8_sweep_70b.log
