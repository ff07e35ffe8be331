# round 4 (o): MoE v3 XCD-contiguous tile order A/B (LLMD_MOE_V3_XCD), numerics with it on
set -o pipefail
mkdir -p gpurun_out
LLMD_MOE_V3_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py tests/test_kernels_gpu.py -q -x -k "moe" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4o_t.log 2>&1 || { tail -5 gpurun_out/r4o_t.log; exit 1; }
tail -1 gpurun_out/r4o_t.log
for x in 0 1 0 1; do
  LLMD_MOE_V3_XCD=$x timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/r4o_b$x.txt 2>&1 || exit $?
  grep -E "T=(4096|5120)" gpurun_out/r4o_b$x.txt | sed "s/^/XCD=$x: /"
done
