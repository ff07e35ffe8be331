# round-3 regression: full GPU test suite, then the bench at the driver's arguments
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r3.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_r3.log
grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests_r3.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "test run aborted rc=$rc"; exit $rc; fi
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3_driver_args.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_r3_driver_args.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_r3_driver_args.log | tail -6 | cut -c1-400
exit $rc
