# round 4 (p): MLA v4 (32-key tiles through a 4-deep LDS ring) numerics and timing vs v3
set -o pipefail
mkdir -p gpurun_out
LLMD_MLA_SHAPE=43 timeout -k 10 300 python -u -m pytest tests/test_deepseek.py tests/test_fp8_kv.py tests/test_kernels_prod_shapes.py -k "mla" -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4p_t.log 2>&1
rc=$?
tail -2 gpurun_out/r4p_t.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r4p_t.log | head; exit $rc; }
for sh in 42 43 42 43; do
  LLMD_MLA_SHAPE=$sh timeout -k 10 150 python -u scripts/bench_attn.py --mla-only > gpurun_out/r4p_b$sh.log 2>&1 || exit $?
  grep "^mla" gpurun_out/r4p_b$sh.log | sed "s/^/shape $sh: /"
done
LLMD_MLA_SHAPE=43 timeout -k 10 300 python -u scripts/bench_mla_split.py > gpurun_out/r4p_split43.log 2>&1 || exit $?
grep rows gpurun_out/r4p_split43.log
