# round 4 (a): new kernel tests (prefill GEMM, masked sampling, LDS copy), the 1-GPU
# multi-rank pre-flight, symm EP (fp8 dispatch), hybrid KV + offload GPU paths,
# then the prefill GEMM A/B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_multi_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "pgemm or sample or kvx or preflight" > gpurun_out/r4a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r4a_tests.log
[ $rc -ne 0 ] && { grep -E "Error|error|FAILED|assert" gpurun_out/r4a_tests.log | head -30; exit $rc; }
timeout -k 10 400 python -u scripts/bench_pgemm.py --rounds 3 > gpurun_out/pgemm_bench.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/pgemm_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_symm.py tests/test_hybrid_kv.py tests/test_offload.py -q -x -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a_tests2.log 2>&1
rc=$?
tail -5 gpurun_out/r4a_tests2.log
[ $rc -ne 0 ] && grep -E "Error|error|FAILED|assert|mismatch|differ" gpurun_out/r4a_tests2.log | head -30
exit $rc
