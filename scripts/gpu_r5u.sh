# Shader clock / package power while the 70B prefill GEMMs run back to back (scripts/gemm_clock_probe.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_clock_probe.py ${ARMS:-gemm} > gpurun_out/r5u_clock_${ARMS:-gemm}.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5u_clock_${ARMS:-gemm}.log | tail -40
exit $rc
