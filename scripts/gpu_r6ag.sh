# fast-reciprocal activation epilogue in the moe8 / moe4 tile kernels: layer A/B, gpt-oss serving, then numerics
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_mxfp4.py > gpurun_out/r6ag_bench.log 2>&1 || { tail -20 gpurun_out/r6ag_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6ag_bench.log | tail -6
for q in fp8 mxfp4; do
timeout -k 10 420 python3 bench.py --model gpt-oss-120b --isl 5150 --osl 250 --quantization $q --concurrency 256 --steps 20 --warmup 5 --fp8-extra off > gpurun_out/r6ag_$q.log 2>&1 || { tail -20 gpurun_out/r6ag_$q.log; exit 1; }
grep '"metric"' gpurun_out/r6ag_$q.log | cut -c1-260
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_moe_mxfp4.py tests/test_fp8_kv.py tests/test_kernels_gpu.py -m gpu -k "gemm8 or v8 or mxfp4 or bf16_v4" > gpurun_out/r6ag_test.log 2>&1 || { tail -40 gpurun_out/r6ag_test.log; exit 1; }
tail -2 gpurun_out/r6ag_test.log
