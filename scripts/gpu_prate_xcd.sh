# 70B prefill-rank rate with the prefill attention XCD remap off / on (interleaved, twice), plus attention tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill" > gpurun_out/attn_tests.log 2>&1 || { echo "attn tests failed"; tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
L=gpurun_out/prate_xcd.log
: > $L
for r in 1 2; do
  for x in 0 1; do
    echo "## LLMD_PREFILL_XCD=$x round $r" >> $L
    LLMD_PREFILL_XCD=$x timeout -k 10 300 python -u scripts/bench_prefill_rate.py --steps 12 >> $L 2>&1 || { echo "prefill rate failed"; tail -20 $L; exit 1; }
  done
done
grep "##\|prefill ISL" $L
