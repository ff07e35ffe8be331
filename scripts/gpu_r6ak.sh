# MXFP4 tile-size threshold: 64-row vs 192 / 256-row tiles around 32-96 rows per expert
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_mxfp4.py 1024,1536,2048,2560,3072 > gpurun_out/r6ak_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6ak_bench.log | tail -8; exit $rc
