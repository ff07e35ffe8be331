# MXFP4 kernel with a 3-buffer LDS stream: numerics (2 / 3 stages, K 2944 / 512), then layer timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_moe_mxfp4.py > gpurun_out/r6ae_test.log 2>&1 || { tail -40 gpurun_out/r6ae_test.log; exit 1; }
tail -2 gpurun_out/r6ae_test.log
timeout -k 10 500 python -u scripts/bench_mxfp4.py > gpurun_out/r6ae_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6ae_bench.log | tail -8; exit $rc
