# final round-6 validation, part 2: the trimmed MXFP4 tests, smoke() and the default bench.py
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_moe_mxfp4.py -m gpu > gpurun_out/r6ao_test.log 2>&1 || { tail -30 gpurun_out/r6ao_test.log; exit 1; }
tail -1 gpurun_out/r6ao_test.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ao_smoke.log 2>&1 || { tail -20 gpurun_out/r6ao_smoke.log; exit 1; }
tail -1 gpurun_out/r6ao_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r6ao_bench.log 2>&1; rc=$?
grep '"metric"' gpurun_out/r6ao_bench.log | cut -c1-400; exit $rc
