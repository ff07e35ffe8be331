# round 4 (ah): final validation of the round-4 tree - full GPU suite, smoke(), the driver bench at its defaults
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4ah_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4ah_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r4ah_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ah_smoke.log 2>&1 || { tail -20 gpurun_out/r4ah_smoke.log; exit 1; }
tail -1 gpurun_out/r4ah_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r4ah_bench.out 2> gpurun_out/r4ah_bench.err || { tail -20 gpurun_out/r4ah_bench.err; exit 1; }
grep "timed step" gpurun_out/r4ah_bench.err | tail -1; tail -1 gpurun_out/r4ah_bench.out | cut -c1-300
