# round 4 (aa): nt (non-temporal) policy on the decode weight stream (mgemm W LDS-DMA, LLMD_MGEMM_NT) and the
# paged-decode K/V loads (LLMD_DECODE_NT): numerics with both on, then 70B decode-only step A/B on one box
set -o pipefail
mkdir -p gpurun_out
LLMD_MGEMM_NT=1 LLMD_DECODE_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_mgemm.py tests/test_kernels_gpu.py -k "decode or mgemm" tests/test_kernels_prod_shapes.py tests/test_fp8_kv.py \
  > gpurun_out/r4aa_tests.log 2>&1 || { tail -30 gpurun_out/r4aa_tests.log; exit 1; }
tail -2 gpurun_out/r4aa_tests.log
for cfg in "0 0" "1 1" "1 0" "0 1" "0 0" "1 1"; do
  set -- $cfg
  LLMD_MGEMM_NT=$1 LLMD_DECODE_NT=$2 timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 60 \
    > gpurun_out/r4aa_d_$1$2.log 2>&1 || { tail -20 gpurun_out/r4aa_d_$1$2.log; exit 1; }
  echo "MGEMM_NT=$1 DECODE_NT=$2: $(grep 'decode batch' gpurun_out/r4aa_d_$1$2.log)" | tee -a gpurun_out/r4aa_summary.txt
done
