# TunableOp search for one rank of a TP2 Llama-3-70B decode replica (M = decode buckets 64/96/128),
# then the TP2-shard decode step with the merged table.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/tune_gemm.py --models llama-3-70b --tp 2 --ms 64 96 128 \
  --names qkv o gate_up down --out gpurun_out/tunableop_tp2.csv > gpurun_out/tune_tp2.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_tp2.log; exit 1; }
grep "default\|total" gpurun_out/tune_tp2.log
cp llmd_amd/tuning/tunableop_gfx950.csv gpurun_out/tunableop_merged.csv
python scripts/merge_tunableop.py gpurun_out/tunableop_merged.csv gpurun_out/tunableop_tp2.csv
cp gpurun_out/tunableop_merged.csv llmd_amd/tuning/tunableop_gfx950.csv
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --tp-shard 2 --batch 128 --steps 30 > gpurun_out/dtp_tuned.log 2>&1 || { echo "decode failed"; tail -20 gpurun_out/dtp_tuned.log; exit 1; }
grep "ms/step\|WARN" gpurun_out/dtp_tuned.log
