# moe8 (fp8 grouped GEMM v8): numerics then v4 vs v8 timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_kv.py -k "v8 or gemm8" > gpurun_out/r6i_test.log 2>&1 || { tail -30 gpurun_out/r6i_test.log; exit 1; }
tail -3 gpurun_out/r6i_test.log
timeout -k 10 300 python -u scripts/bench_moe8.py > gpurun_out/r6i_bench.log 2>&1; rc=$?
cat gpurun_out/r6i_bench.log; exit $rc
