# persistent cross-tile pgemm (variant 6) numerics + A/B vs variant 3 and hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "pgemm" > gpurun_out/r5d_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5d_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u scripts/bench_pgemm.py --rounds 3 --ms 4608,8192,2048 --shapes qkv,o,gate_up,down,8b_qkv,8b_gate_up --variants 3,6 > gpurun_out/r5d_pgemm.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5d_pgemm.log | tail -18
exit $rc
