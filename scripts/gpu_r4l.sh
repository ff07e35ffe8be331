# round 4 (l): fp8 MoE v3 schedule A/B on one box (LLMD_MOE_V3_VARIANT: bit 0 = A fragments one
# block ahead, bit 1 = asm LDS-DMA), numerics of each variant first
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3; do
  LLMD_MOE_V3_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py -q -x -k "moe_fp8_prefill_tiles" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4l_t$v.log 2>&1 || { echo "variant $v tests failed"; tail -5 gpurun_out/r4l_t$v.log; exit 1; }
  LLMD_MOE_V3_VARIANT=$v timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/r4l_b$v.txt 2>&1 || exit $?
  grep -E "T=(4096|5120)" gpurun_out/r4l_b$v.txt | sed "s/^/V=$v: /"
done
