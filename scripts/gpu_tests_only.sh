# full GPU test suite only (no bench); log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -20
exit $rc
