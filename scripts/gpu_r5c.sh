# pgemm variant 3 schedule A/B: 3 (reads from MFMA 37), 4 (+ sc1 DMA), 5 (reads from MFMA 44)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/bench_pgemm.py --rounds 3 --ms 4608,518 --shapes qkv,o,gate_up,down,8b_qkv,8b_gate_up,8b_down --variants 3,4,5 > gpurun_out/r5c_pgemm.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5c_pgemm.log | tail -16
exit $rc
