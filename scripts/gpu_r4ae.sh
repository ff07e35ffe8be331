# round 4 (ae): medium-M decode GEMM plan sweep with the nt weight stream (70B TP1 M 64/128, TP2 shard M 64/128)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/sweep_mgemm.py --model llama-3-70b --tp 1 --m 64 128 > gpurun_out/r4ae_sweep_tp1.log 2>&1 || { echo "sweep tp1 failed"; tail -20 gpurun_out/r4ae_sweep_tp1.log; exit 1; }
grep "hipBLASLt\|WRONG" gpurun_out/r4ae_sweep_tp1.log
timeout -k 10 400 python -u scripts/sweep_mgemm.py --model llama-3-70b --tp 2 --m 64 128 > gpurun_out/r4ae_sweep_tp2.log 2>&1 || { echo "sweep tp2 failed"; tail -20 gpurun_out/r4ae_sweep_tp2.log; exit 1; }
grep "hipBLASLt\|WRONG" gpurun_out/r4ae_sweep_tp2.log
