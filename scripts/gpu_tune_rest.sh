# TunableOp for remaining serving shapes: Llama-3-8B 512-aligned mixed steps + decode buckets, the Qwen3-32B
# and gpt-oss-120b LM heads at decode batch sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/tune_gemm.py --models llama-3-8b --ms 96 160 256 512 1024 1536 2048 3072 4096 4608 --names qkv o gate_up down --out gpurun_out/tunableop_8b.csv > gpurun_out/tune_8b.log 2>&1 || { tail -20 gpurun_out/tune_8b.log; exit 1; }
grep "total" gpurun_out/tune_8b.log
timeout -k 10 600 python -u scripts/tune_gemm.py --models qwen3-32b gpt-oss-120b --ms 1 8 16 32 64 128 256 --names lm_head --out gpurun_out/tunableop_lmh.csv > gpurun_out/tune_lmh.log 2>&1 || { tail -20 gpurun_out/tune_lmh.log; exit 1; }
grep "M=\|total" gpurun_out/tune_lmh.log
