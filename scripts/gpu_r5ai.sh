# Medium-M decode GEMM plan sweep for Llama-3-8B TP1 (M 64 / 96 / 128), cold weights, vs hipBLASLt + stream kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/sweep_mgemm.py --model llama-3-8b --tp 1 --m 64 96 128 > gpurun_out/mgemm_sweep_8b_tp1.log 2>&1
rc=$?; grep -c "^ROW" gpurun_out/mgemm_sweep_8b_tp1.log; tail -3 gpurun_out/mgemm_sweep_8b_tp1.log; exit $rc
