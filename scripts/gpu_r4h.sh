# round 4 (h): MLA v3 (literal-AGPR accumulators) numerics, then timing vs v2
set -o pipefail
mkdir -p gpurun_out
LLMD_MLA_SHAPE=42 timeout -k 10 300 python -u -m pytest tests/test_deepseek.py tests/test_fp8_kv.py tests/test_kernels_prod_shapes.py -k mla -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/mla42_tests.log 2>&1
rc=$?
tail -3 gpurun_out/mla42_tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" gpurun_out/mla42_tests.log | head -20; exit $rc; }
for sh in 42 41; do
  LLMD_MLA_SHAPE=$sh timeout -k 10 150 python -u scripts/bench_attn.py --mla-only > gpurun_out/mla_shape_$sh.log 2>&1 || exit $?
  grep "^mla" gpurun_out/mla_shape_$sh.log | sed "s/^/shape $sh: /"
  LLMD_MLA_SHAPE=$sh timeout -k 10 150 python -u scripts/bench_attn.py --mla-only --kv-dtype fp8 > gpurun_out/mla_shape_${sh}_fp8.log 2>&1 || exit $?
  grep "^mla" gpurun_out/mla_shape_${sh}_fp8.log | sed "s/^/shape $sh: /"
done
