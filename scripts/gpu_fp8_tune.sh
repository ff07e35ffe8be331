# fp8 W8A8 projections of Llama-3-70B: TunableOp over hipBLASLt's scaled GEMMs (row-wise scales), then the
# fp8-weights + fp8-KV decode step before / after merging the results into this box's copy of the table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --batch 64 --isl 5000 --steps 30 2>&1 | grep "ms/step" | sed 's/^/before: /' || exit 1
timeout -k 10 900 python -u scripts/tune_fp8_gemm.py --models llama-3-70b --ms 1 16 32 64 128 256 512 4608 --out gpurun_out/tunableop_fp8.csv > gpurun_out/tune_fp8.log 2>&1 || { tail -20 gpurun_out/tune_fp8.log; exit 1; }
grep "M=\|total" gpurun_out/tune_fp8.log
grep -c "ScaledGemm" gpurun_out/tunableop_fp8.csv || { echo "no scaled-GEMM entries recorded"; exit 0; }
python scripts/merge_tunableop.py llmd_amd/tuning/tunableop_gfx950.csv gpurun_out/tunableop_fp8.csv
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --batch 64 --isl 5000 --steps 30 2>&1 | grep "ms/step" | sed 's/^/after: /' || exit 1
