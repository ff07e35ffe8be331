set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "moe" --timeout 120 --timeout-method thread > gpurun_out/moe2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/moe2_tests.log; exit 1; }
tail -1 gpurun_out/moe2_tests.log
LLMD_MOE_GEMM_V1=1 timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_v1.txt 2>&1 && timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_v2.txt 2>&1 || { echo bench failed; tail gpurun_out/moe_v2.txt; exit 1; }
echo "== v1"; grep -v amdgpu gpurun_out/moe_v1.txt; echo "== v2"; grep -v amdgpu gpurun_out/moe_v2.txt
