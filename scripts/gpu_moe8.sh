set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/moe8_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/moe8_tests.log; exit 1; }
tail -1 gpurun_out/moe8_tests.log
timeout -k 10 300 python scripts/bench_moe.py > gpurun_out/moe_fp8_bench.txt 2>&1 || { echo bench failed; tail -20 gpurun_out/moe_fp8_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/moe_fp8_bench.txt
