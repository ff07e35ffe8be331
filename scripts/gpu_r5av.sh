# Bench after the host-side metric batching (EPP + engine ITL/TTFT) and the GPU engine tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_engine.py tests/test_router_metrics_deferred.py > gpurun_out/r5av_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5av_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r5av_bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5av_bench.log | tail -12; exit $rc
