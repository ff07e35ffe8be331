# TunableOp search for the step sizes the N=1 bench's closed loop really produces (timed step-size histogram:
# 4608 = 512-aligned first chunk, 518 = prompt remainder + 64 decode rows; 576 = that remainder padded to 64).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/tune_gemm.py --models llama-3-70b --ms 518 576 4608 \
  --names qkv o gate_up down --duration-ms 20 --out gpurun_out/tunableop_steps.csv > gpurun_out/tune_steps.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_steps.log; exit 1; }
grep "default\|total" gpurun_out/tune_steps.log
