# Full GPU suite (as the driver runs it) + smoke() on the current tree.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r5al_gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5al_gpu_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5al_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r5al_smoke.log; exit $rc
