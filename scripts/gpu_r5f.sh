# v6 numerics + A/B (incl. M 5064), kvx copy-engine A/B, then the offline prefill-GEMM table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "pgemm" > gpurun_out/r5f_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5f_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_pgemm.py --rounds 3 --ms 4608,5064,518 --shapes qkv,o,gate_up,down --variants 3,6 > gpurun_out/r5f_pgemm.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5f_pgemm.log | grep "^M="
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench/kvx_copy_ab.py --rounds 5 > gpurun_out/r5f_kvx_ab.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5f_kvx_ab.log | tail -34
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/make_pgemm_table.py --rounds 3 --variants 0,3,6 --models 70b,8b,70b_tp2 --out gpurun_out/pgemm_table.py > gpurun_out/r5f_table.log 2>&1
rc=$?
tail -3 gpurun_out/r5f_table.log
exit $rc
