# moe8 persistent fp8 grouped GEMM: numerics, then v4 vs v8 timing and per-tile fixed cost
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_kv.py -k "v8 or gemm8" > gpurun_out/r6k_test.log 2>&1 || { tail -40 gpurun_out/r6k_test.log; exit 1; }
tail -3 gpurun_out/r6k_test.log
timeout -k 10 300 python -u scripts/bench_moe8.py > gpurun_out/r6k_bench.log 2>&1 || { cat gpurun_out/r6k_bench.log; exit 1; }
cat gpurun_out/r6k_bench.log
VERS=4,8 timeout -k 10 300 python -u scripts/moe_tile_overhead.py > gpurun_out/r6k_ovh.log 2>&1; rc=$?
cat gpurun_out/r6k_ovh.log; exit $rc
