# MXFP4 experts on 64-row tiles for decode-sized steps: numerics (kernel + layer), then layer timing A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_moe_mxfp4.py -m gpu > gpurun_out/r6aj_test.log 2>&1 || { tail -40 gpurun_out/r6aj_test.log; exit 1; }
tail -2 gpurun_out/r6aj_test.log
timeout -k 10 400 python -u scripts/bench_mxfp4.py > gpurun_out/r6aj_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6aj_bench.log | tail -8; exit $rc
