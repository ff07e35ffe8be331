# MXFP4 tile GEMM K-step decomposition (diagnostic variants, garbage outputs by design)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/mxfp4_diag.py > gpurun_out/r6as.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6as.log | tail -4; exit $rc
