# round 4 (ad): nt policy on the MoE v3 expert-weight DMA (LLMD_MOE_V3_NT) - numerics, then bench_moe A/B (0 1 0 1)
set -o pipefail
mkdir -p gpurun_out
LLMD_MOE_V3_NT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "moe" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4ad_t.log 2>&1 || { tail -20 gpurun_out/r4ad_t.log; exit 1; }
tail -1 gpurun_out/r4ad_t.log
for v in 0 1 0 1; do
  LLMD_MOE_V3_NT=$v timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/r4ad_b$v.txt 2>&1 || exit $?
  grep -E "T=(4096|5120)" gpurun_out/r4ad_b$v.txt | sed "s/^/V3_NT=$v: /" | tee -a gpurun_out/r4ad_summary.txt
done
