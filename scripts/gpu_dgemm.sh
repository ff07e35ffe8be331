# Decode GEMM: numerics tests, then the plan sweep (70B and 8B shapes) against hipBLASLt+TunableOp.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dgemm_tests.log 2>&1 || { echo "dgemm tests failed"; tail -40 gpurun_out/dgemm_tests.log; exit 1; }
tail -1 gpurun_out/dgemm_tests.log
for m in llama-3-70b llama-3-8b; do
  timeout -k 10 600 python -u scripts/sweep_dgemm.py --model $m --m 1 8 16 32 48 64 > gpurun_out/dgemm_sweep_$m.log 2>&1 || { echo "sweep failed"; tail -30 gpurun_out/dgemm_sweep_$m.log; exit 1; }
  grep -v "^   top5\|^ROW\|amdgpu.ids" gpurun_out/dgemm_sweep_$m.log | cut -c1-160
done
