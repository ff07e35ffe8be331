# K-step-major MXFP4 scales too: numerics both layouts, engine test, layer A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_moe_mxfp4.py tests/test_engine.py -m gpu -k "mxfp4" > gpurun_out/r6ax_test.log 2>&1 || { tail -40 gpurun_out/r6ax_test.log; exit 1; }
tail -1 gpurun_out/r6ax_test.log
timeout -k 10 400 python -u scripts/bench_mxfp4.py 256,1024,2048,5405,8192 > gpurun_out/r6ax_bench.log 2>&1 || { tail -20 gpurun_out/r6ax_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6ax_bench.log | tail -6
timeout -k 10 300 python -u scripts/mxfp4_diag.py > gpurun_out/r6ax_diag.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6ax_diag.log | tail -3; exit $rc
