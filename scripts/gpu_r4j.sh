# round 4 (j): MLA with bf16 partials + the vectorised merge (defaults now) - numerics and timing,
# then the DeepSeek-R1 one-EP-rank projection (scripts/gpu_r4b.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_deepseek.py tests/test_fp8_kv.py tests/test_kernels_prod_shapes.py -k "mla" -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4j_mla_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4j_mla_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r4j_mla_tests.log | head; exit $rc; }
timeout -k 10 150 python -u scripts/bench_attn.py --mla-only > gpurun_out/r4j_mla.log 2>&1 || exit $?
grep "^mla" gpurun_out/r4j_mla.log
timeout -k 10 150 python -u scripts/bench_attn.py --mla-only --kv-dtype fp8 > gpurun_out/r4j_mla_fp8.log 2>&1 || exit $?
grep "^mla" gpurun_out/r4j_mla_fp8.log
bash scripts/gpu_r4b.sh
