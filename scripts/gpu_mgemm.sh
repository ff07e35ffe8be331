# Medium-M decode GEMM: numerics tests, then plan sweeps (70B TP1 and TP2-shard shapes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mgemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mgemm_test.log 2>&1 || { echo "mgemm tests failed"; tail -30 gpurun_out/mgemm_test.log; exit 1; }
tail -2 gpurun_out/mgemm_test.log
timeout -k 10 400 python -u scripts/sweep_mgemm.py --model llama-3-70b --tp 2 --m 64 96 128 > gpurun_out/mgemm_sweep_70b_tp2.log 2>&1 || { echo "sweep tp2 failed"; tail -20 gpurun_out/mgemm_sweep_70b_tp2.log; exit 1; }
grep "hipBLASLt\|WRONG" gpurun_out/mgemm_sweep_70b_tp2.log
timeout -k 10 400 python -u scripts/sweep_mgemm.py --model llama-3-70b --tp 1 --m 64 128 > gpurun_out/mgemm_sweep_70b_tp1.log 2>&1 || { echo "sweep tp1 failed"; tail -20 gpurun_out/mgemm_sweep_70b_tp1.log; exit 1; }
grep "hipBLASLt\|WRONG" gpurun_out/mgemm_sweep_70b_tp1.log
