# After the decode reduce fusions: P/D same-device greedy checks, engine tests, then the driver bench twice.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_pd_cross_device.py tests/test_pd_gpu.py tests/test_models_gpu.py tests/test_tp.py -m gpu > gpurun_out/r5ae_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5ae_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ae_bench$i.log 2>&1
  rc=$?; grep -E "timed step sizes" gpurun_out/r5ae_bench$i.log; grep -o '"value": [0-9.]*' gpurun_out/r5ae_bench$i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
