# MXFP4 64-row tiles at decode sizes: 2 vs 3 LDS K-step buffers (latency-bound K-steps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_mxfp4.py 64,256,1024 > gpurun_out/r6am_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6am_bench.log | tail -8; exit $rc
