# fp8 grouped GEMM v3 (256-row expert tiles): numerics, then the MoE microbenchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_kv.py -x -q --timeout 120 --timeout-method thread -k "moe" > gpurun_out/moe_v3_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/moe_v3_tests.log; exit 1; }
tail -1 gpurun_out/moe_v3_tests.log
timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_v3_bench.txt 2>&1 || { echo bench failed; tail -20 gpurun_out/moe_v3_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/moe_v3_bench.txt
