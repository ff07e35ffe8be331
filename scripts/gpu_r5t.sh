# The whole GPU suite as the driver runs it (pytest -m gpu), per-test timeout, no -x so every failure shows.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r5t_gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5t_gpu_tests.log | tail -30
exit $rc
