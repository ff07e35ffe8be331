# round 4 (n): bf16 MoE v3 schedule A/B (LLMD_MOE_V3_BF16_VARIANT), then the driver's bench at its defaults
set -o pipefail
mkdir -p gpurun_out
for v in 2 3; do
  LLMD_MOE_V3_BF16_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "moe_experts" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4n_t$v.log 2>&1 || { echo "variant $v tests failed"; tail -5 gpurun_out/r4n_t$v.log; exit 1; }
  LLMD_MOE_V3_BF16_VARIANT=$v timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/r4n_b$v.txt 2>&1 || exit $?
  grep -E "T=(4096|5120)" gpurun_out/r4n_b$v.txt | sed "s/^/BFV=$v: /"
done
timeout -k 10 900 python -u bench.py > gpurun_out/r4n_bench.out 2> gpurun_out/r4n_bench.err || { tail -20 gpurun_out/r4n_bench.err; exit 1; }
grep "timed step" gpurun_out/r4n_bench.err | tail -1
tail -1 gpurun_out/r4n_bench.out
