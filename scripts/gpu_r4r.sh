# round 4 (r): GQA prefill v2 read-ahead A/B (LLMD_PREFILL_V2_VARIANT 1 = ring PF 4, 5 = PF 6, 9 = first V
# fragments before the softmax, 13 = both), numerics of each first
set -o pipefail
mkdir -p gpurun_out
for v in 1 5 9 13 1; do
  LLMD_PREFILL_V2_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "paged_prefill" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4r_t$v.log 2>&1 || { echo "variant $v tests failed"; tail -5 gpurun_out/r4r_t$v.log; exit 1; }
  LLMD_PREFILL_V2_VARIANT=$v timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/r4r_b$v.txt 2>&1 || exit $?
  grep -E "^prefill ctx=(5000|8192)" gpurun_out/r4r_b$v.txt | sed "s/^/V=$v: /"
done
