# final tree check: smoke() and the MXFP4 engine / weight tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6az_smoke.log 2>&1 || { tail -20 gpurun_out/r6az_smoke.log; exit 1; }
tail -1 gpurun_out/r6az_smoke.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine.py tests/test_weight_sync.py -m gpu > gpurun_out/r6az_test.log 2>&1; rc=$?
tail -1 gpurun_out/r6az_test.log; exit $rc
