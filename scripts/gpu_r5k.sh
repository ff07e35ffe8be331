# MoE v4 192-row tiles with 64 KB-aligned buffers: error maps at K = 64, 128, 1024
set -o pipefail
mkdir -p gpurun_out
for dd in 128; do
  DIAG_D=$dd timeout -k 10 300 python -u scripts/moe4_diag.py 192 > gpurun_out/r5k_diag192_$dd.log 2>&1
  rc=$?; echo "== K=$dd"; grep -v amdgpu.ids gpurun_out/r5k_diag192_$dd.log | grep -E "gather|slots|mode1|fp8|bad fraction per 16-row" | head -7; [ $rc -ne 0 ] && exit $rc
done
exit 0
