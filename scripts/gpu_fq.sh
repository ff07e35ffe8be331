set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fq_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fq_tests.log; exit 1; }
tail -1 gpurun_out/fq_tests.log
timeout -k 10 300 python scripts/bench_decode.py --quantization fp8 --kv-cache-dtype fp8 --steps 30 > gpurun_out/fq_decode.txt 2>&1 || { echo "bench failed"; tail -20 gpurun_out/fq_decode.txt; exit 1; }
grep decode gpurun_out/fq_decode.txt
