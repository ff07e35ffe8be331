# prefill GEMM: numerics tests, masked-row sampling test, then the A/B bench vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "pgemm or sample" > gpurun_out/pgemm_tests.log 2>&1
rc=$?
tail -5 gpurun_out/pgemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_pgemm.py --rounds 3 > gpurun_out/pgemm_bench.log 2>&1
rc=$?
cat gpurun_out/pgemm_bench.log | grep -v amdgpu.ids
exit $rc
