# fp8 group quant as one wave per row: numerics (fp8 / MoE / W8A8), MoE A/B, gpt-oss serving.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_fp8_kv.py tests/test_kernels_gpu.py tests/test_models_gpu.py -k "moe or gpt or fp8 or quant" > gpurun_out/r5at_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5at_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_moe.py > gpurun_out/r5at_moe.log 2>&1
rc=$?; grep -E "T=4096|T=5120" gpurun_out/r5at_moe.log; [ $rc -ne 0 ] && exit $rc
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10 --quantization fp8 --concurrency 256"
timeout -k 10 500 python -u bench.py $M > gpurun_out/r5at_gptoss.log 2>&1
rc=$?; grep -E "timed step sizes" gpurun_out/r5at_gptoss.log; grep -o '"value": [0-9.]*' gpurun_out/r5at_gptoss.log; exit $rc
