# Final round-5 validation after the metric batching on the current tree: the full GPU suite (as the driver runs it), smoke(), the driver bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r5ax_gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5ax_gpu_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5ax_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r5ax_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ax_bench.log 2>&1
rc=$?; grep -E "timed step sizes" gpurun_out/r5ax_bench.log; grep '^{' gpurun_out/r5ax_bench.log | cut -c1-200; exit $rc
