# MoE v4 bf16 error map (scripts/moe4_diag.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/moe4_diag.py > gpurun_out/r5k_diag.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5k_diag.log | head -80; exit $rc
