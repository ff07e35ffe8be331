# Decode GEMM: tests, then load-path variants (LLMD_DGEMM_VAR: 2 rotated k start) vs baseline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dgemm_tests.log 2>&1 || { echo "dgemm tests failed"; tail -40 gpurun_out/dgemm_tests.log; exit 1; }
tail -1 gpurun_out/dgemm_tests.log
for v in 0 2; do
  LLMD_DGEMM_VAR=$v timeout -k 10 300 python -u scripts/sweep_dgemm.py --model llama-3-70b --m 64 16 > gpurun_out/dgemm_var$v.log 2>&1 || { echo "var $v failed"; tail -20 gpurun_out/dgemm_var$v.log; exit 1; }
  echo "== VAR $v"; grep -v "amdgpu.ids" gpurun_out/dgemm_var$v.log | cut -c1-150
done
