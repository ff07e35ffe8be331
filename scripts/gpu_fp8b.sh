set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8b_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fp8b_tests.log; exit 1; }
tail -1 gpurun_out/fp8b_tests.log
for args in "--kv-cache-dtype fp8" "--quantization fp8 --kv-cache-dtype fp8" "--quantization fp8 --kv-cache-dtype fp8 --batch 128"; do
  timeout -k 10 300 python scripts/bench_decode.py $args --steps 30 >> gpurun_out/fp8_decode.txt 2>&1 || { echo "bench failed: $args"; tail -20 gpurun_out/fp8_decode.txt; exit 1; }
done
grep decode gpurun_out/fp8_decode.txt
