# round 4 (t): GEMM time around M = 518 (the 455-token prompt remainder + 63 decode rows step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_pgemm.py --ms 512,518,576,640,1024 --shapes qkv,o,gate_up,down --rounds 2 > gpurun_out/r4t_pgemm.txt 2>&1 || exit $?
grep "^M=" gpurun_out/r4t_pgemm.txt
