# pgemm variant 3 (PGR2 LDS-DMA, whole K-step in registers) A/B + PMC vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_pgemm.py --rounds 3 --ms 4608 --shapes qkv,o,gate_up,down,8b_qkv --variants 0,3 > gpurun_out/r5b_pgemm.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5b_pgemm.log | tail -12
[ $rc -ne 0 ] && exit $rc
PGEMM_PMC_ARGS="--variants 0,3" bash scripts/gpu_pgemm_pmc.sh
