# fp8 experts on 64-row persistent tiles for decode-sized steps: numerics, then decode-size timing A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp8_kv.py -m gpu -k "t64 or gemm8_fp8_kernel or (v8 and 2880)" > gpurun_out/r6al_test.log 2>&1 || { tail -40 gpurun_out/r6al_test.log; exit 1; }
tail -2 gpurun_out/r6al_test.log
timeout -k 10 400 python -u scripts/bench_moe_decode.py > gpurun_out/r6al_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6al_bench.log | tail -12; exit $rc
