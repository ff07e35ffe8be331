# fp8-KV prefill through the bf16 copy: numerics, then the fp8 serving bench (70B) with it on / off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp8_kv.py -k "prefill_fp8 or dequant" > gpurun_out/r6z_test.log 2>&1 || { tail -40 gpurun_out/r6z_test.log; exit 1; }
tail -2 gpurun_out/r6z_test.log
for m in 1 0; do
  LLMD_PREFILL_FP8_VIA_BF16=$m timeout -k 10 600 python -u bench.py --quantization fp8 --kv-cache-dtype fp8 --fp8-extra off --steps 20 --warmup 5 > gpurun_out/r6z_bench_$m.log 2>&1 || { tail -20 gpurun_out/r6z_bench_$m.log; exit 1; }
  echo "via_bf16=$m"; grep '"metric"' gpurun_out/r6z_bench_$m.log | cut -c1-420
done
