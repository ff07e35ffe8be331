# Qwen3-32B decode GEMMs: small-M stream kernel sweep, then the decode step A/B with the medium-M
# LDS-DMA kernel table entries (LLMD_SKINNY_GEMM=0 = hipBLASLt + TunableOp everywhere)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/sweep_dgemm.py --model qwen3-32b --m 16 32 64 --quick > gpurun_out/dgemm_sweep_qwen3_32b.log 2>&1 || { echo "dgemm sweep failed"; tail -20 gpurun_out/dgemm_sweep_qwen3_32b.log; exit 1; }
grep -v "^ROW\|amdgpu.ids" gpurun_out/dgemm_sweep_qwen3_32b.log | tail -14
for b in 64 128; do
  for sk in 0 1; do
    LLMD_SKINNY_GEMM=$sk timeout -k 10 300 python -u scripts/bench_decode.py --model qwen3-32b --batch $b --isl 2000 --steps 40 2>&1 | grep -v amdgpu.ids | grep "ms/step" | sed "s/^/skinny=$sk /" || exit 1
  done
done
