# TunableOp for the remaining serving shapes: Qwen3-32B decode buckets and 512-aligned mixed steps, Llama-3-70B
# aligned prefill steps missing from the table (2560 / 3072 / 4608)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/tune_gemm.py --models qwen3-32b --ms 1 2 4 8 16 32 64 96 128 160 256 1536 2048 3072 4096 4608 6144 8192 --names qkv o gate_up down --out gpurun_out/tunableop_q32b.csv > gpurun_out/tune_q32b.log 2>&1 || { tail -20 gpurun_out/tune_q32b.log; exit 1; }
grep "total" gpurun_out/tune_q32b.log
timeout -k 10 600 python -u scripts/tune_gemm.py --models llama-3-70b --ms 2560 3072 4608 --names qkv o gate_up down --out gpurun_out/tunableop_70b.csv > gpurun_out/tune_70b.log 2>&1 || { tail -20 gpurun_out/tune_70b.log; exit 1; }
grep "M=\|total" gpurun_out/tune_70b.log
