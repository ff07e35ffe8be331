# MoE v4 192-row tiles after the per-iteration drain: error maps at K = 64, 128, 1024 and the MoE tests at both tiles
set -o pipefail
mkdir -p gpurun_out
for dd in 64 128 1024; do
  DIAG_D=$dd timeout -k 10 300 python -u scripts/moe4_diag.py 192 > gpurun_out/r5k_diag192_$dd.log 2>&1
  rc=$?; echo "== K=$dd"; grep -v amdgpu.ids gpurun_out/r5k_diag192_$dd.log | grep -E "gather|slots|mode1|fp8|bad fraction per 16-row" | head -7; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_kv.py -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "moe" > gpurun_out/r5k_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5k_tests.log; exit $rc
