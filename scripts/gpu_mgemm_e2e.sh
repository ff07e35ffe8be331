# Decode step with the medium-M decode GEMM table vs hipBLASLt only (LLMD_SKINNY_GEMM=0):
# 70B TP1 batch 64 and one TP2-shard rank at batch 96 / 128.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/mgemm_e2e.log
: > $L
run() { timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b "$@" --steps 30 >> $L 2>&1 || { echo "decode $* failed"; tail -20 $L; exit 1; }; }
echo "## mgemm+stream tables" >> $L
run --batch 64
run --tp-shard 2 --batch 128
run --tp-shard 2 --batch 96
echo "## hipBLASLt only" >> $L
export LLMD_SKINNY_GEMM=0
run --batch 64
run --tp-shard 2 --batch 128
grep "##\|ms/step\|WARN" $L
