# round 5 first GPU call: the new GPU tests (stalled-peer, offload, hybrid, symm) and the
# prefill GEMM A/B with the register-staged variant 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_collective_failure.py tests/test_symm.py tests/test_offload.py tests/test_hybrid_kv.py \
  > gpurun_out/r5a_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r5a_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u scripts/bench_pgemm.py --rounds 3 --ms 4608,518 --variants 0,2 > gpurun_out/r5a_pgemm.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5a_pgemm.log
exit $rc
