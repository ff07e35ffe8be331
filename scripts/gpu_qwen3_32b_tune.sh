# Qwen3-32B decode path: qk-norm kernel numerics, then decode GEMM plan sweeps at its shapes
# (medium-M LDS-DMA kernel M 64/96/128 and the small-M stream kernel M 16/32/64).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "qk_rms_norm or rms_norm" --timeout 120 --timeout-method thread > gpurun_out/qknorm_test.log 2>&1 || { echo "qk norm tests failed"; tail -30 gpurun_out/qknorm_test.log; exit 1; }
tail -1 gpurun_out/qknorm_test.log
timeout -k 10 400 python -u scripts/sweep_mgemm.py --model qwen3-32b --tp 1 --m 64 96 128 > gpurun_out/mgemm_sweep_qwen3_32b_tp1.log 2>&1 || { echo "mgemm sweep failed"; tail -20 gpurun_out/mgemm_sweep_qwen3_32b_tp1.log; exit 1; }
grep "hipBLASLt\|WRONG" gpurun_out/mgemm_sweep_qwen3_32b_tp1.log | head -20
timeout -k 10 400 python -u scripts/sweep_dgemm.py --model qwen3-32b --m 16 32 64 --quick > gpurun_out/dgemm_sweep_qwen3_32b.log 2>&1 || { echo "dgemm sweep failed"; tail -20 gpurun_out/dgemm_sweep_qwen3_32b.log; exit 1; }
tail -15 gpurun_out/dgemm_sweep_qwen3_32b.log
