# persistent pgemm (variant 6) numerics + A/B, then the kvx copy-engine A/B
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_r5d.sh || exit $?
timeout -k 10 300 python -u bench/kvx_copy_ab.py --rounds 5 > gpurun_out/r5e_kvx_ab.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5e_kvx_ab.log | tail -40
exit $rc
