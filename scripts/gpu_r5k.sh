# MoE v4 error maps at both tile sizes (scripts/moe4_diag.py), then the MoE tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/moe4_diag.py 192 > gpurun_out/r5k_diag192.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5k_diag192.log | head -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/moe4_diag.py 256 > gpurun_out/r5k_diag256.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5k_diag256.log | head -12
exit $rc
