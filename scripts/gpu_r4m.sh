# round 4 (m): GQA prefill v2 schedule A/B on one box (LLMD_PREFILL_V2_VARIANT: bit 0 = ring-pipelined
# fragment reads with sched_barriers, bit 1 = asm LDS-DMA), numerics of each variant first
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3 3 0; do
  LLMD_PREFILL_V2_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "paged_prefill" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4m_t$v.log 2>&1 || { echo "variant $v tests failed"; tail -5 gpurun_out/r4m_t$v.log; exit 1; }
  LLMD_PREFILL_V2_VARIANT=$v timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/r4m_b$v.txt 2>&1 || exit $?
  grep -E "^prefill ctx=(5000|8192)" gpurun_out/r4m_b$v.txt | sed "s/^/V=$v: /"
done
