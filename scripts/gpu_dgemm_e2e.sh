# Decode GEMM in the engine: GPU tests, then decode-step A/B (table dispatch vs hipBLASLt only).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
for m in llama-3-8b; do for b in 8 32 64; do for v in 0 1; do
  LLMD_SKINNY_GEMM=$v timeout -k 10 300 python scripts/bench_decode.py --model $m --batch $b --isl 2000 --steps 40 > gpurun_out/dec_${m}_${b}_$v.log 2>&1 || { echo "decode bench failed"; tail -20 gpurun_out/dec_${m}_${b}_$v.log; exit 1; }
  echo "skinny=$v $(grep -h 'ms/step' gpurun_out/dec_${m}_${b}_$v.log | tail -1)"
done; done; done
for b in 8 64; do for v in 0 1; do
  LLMD_SKINNY_GEMM=$v timeout -k 10 400 python scripts/bench_decode.py --model llama-3-70b --batch $b --isl 5000 --steps 30 > gpurun_out/dec_70b_${b}_$v.log 2>&1 || { echo "decode bench failed"; tail -20 gpurun_out/dec_70b_${b}_$v.log; exit 1; }
  echo "skinny=$v $(grep -h 'ms/step' gpurun_out/dec_70b_${b}_$v.log | tail -1)"
done; done
