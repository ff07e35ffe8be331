# round 4 (a): new kernel tests (prefill GEMM, masked sampling, LDS copy), the 1-GPU
# multi-rank pre-flight, then the prefill GEMM A/B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 360 python -u -m pytest tests/test_kernels_gpu.py tests/test_multi_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "pgemm or sample or kvx or preflight" > gpurun_out/r4a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r4a_tests.log
[ $rc -ne 0 ] && { grep -E "Error|error|FAILED|assert" gpurun_out/r4a_tests.log | head -30; exit $rc; }
timeout -k 10 360 python -u scripts/bench_pgemm.py --rounds 3 > gpurun_out/pgemm_bench.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/pgemm_bench.log
exit $rc
