# Round 6: fp8 GEMM split-K tests, clock/power, the offline fp8 table, fp8 prefill rate + profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_pgemm_fp8.py > gpurun_out/r6c_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_pgemm_fp8.py --m 4608,5063,8192 > gpurun_out/r6c_pgemm8.log 2>&1
rc=$?; cat gpurun_out/r6c_pgemm8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_pgemm_fp8.py --m 5063 --shapes gate_up,down --power > gpurun_out/r6c_pgemm8_power.log 2>&1
rc=$?; grep -v "^GPU\|^=\|^$\|Mhz\|^Device" gpurun_out/r6c_pgemm8_power.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/make_pgemm8_table.py > gpurun_out/r6c_table.log 2>&1
rc=$?; tail -3 gpurun_out/r6c_table.log; [ $rc -eq 0 ] || exit $rc
cp llmd_amd/ops/pgemm8_table.py gpurun_out/pgemm8_table.py
for q in bf16 fp8; do
  extra=""; [ $q = fp8 ] && extra="--quantization fp8"
  timeout -k 10 300 python -u scripts/bench_prefill_rate.py $extra > gpurun_out/r6c_prate_$q.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r6c_prate_$q.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
