# round 4 (w): the full GPU suite again with the rebuilt debug op library (_C_debug) in tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4w_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4w_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r4w_gpu_tests.log | head -20; exit $rc; }
exit 0
