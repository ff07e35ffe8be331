# Prefill attention XCD-aware workgroup remap: numerics tests, then the microbenchmark off/on, twice interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_kv.py -x -q --timeout 120 --timeout-method thread -k "prefill or attention or window" > gpurun_out/attn_tests.log 2>&1 || { echo "attn tests failed"; tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for r in 1 2; do
  for x in 0 1; do
    echo "## LLMD_PREFILL_XCD=$x round $r"
    LLMD_PREFILL_XCD=$x timeout -k 10 300 python -u scripts/bench_attn.py --check > gpurun_out/attn_xcd_$x.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attn_xcd_$x.log; exit 1; }
    grep "prefill" gpurun_out/attn_xcd_$x.log | grep -v "Hq=16"
  done
done
