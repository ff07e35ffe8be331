# MXFP4 vs fp8 gpt-oss MoE layer timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/bench_mxfp4.py > gpurun_out/r6ac_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6ac_bench.log | tail -8; exit $rc
