# Medium-M decode GEMM plan sweep for Llama-3-70B TP4 (the reference AMD recipe's decode TP) (M 64 / 96 / 128), cold weights, vs hipBLASLt + stream kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/sweep_mgemm.py --model llama-3-70b --tp 4 --m 64 96 128 > gpurun_out/mgemm_sweep_70b_tp4.log 2>&1
rc=$?; grep -c "^ROW" gpurun_out/mgemm_sweep_70b_tp4.log; tail -3 gpurun_out/mgemm_sweep_70b_tp4.log; exit $rc
