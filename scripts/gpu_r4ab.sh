# round 4 (ab): nt policy on the v2 MoE expert-weight stream (LLMD_MOE_NT) - numerics, gpt-oss-120b decode-only
# A/B (fp8 batch 256, bf16 batch 112, ISL 5150), then the driver's 70B bench at its defaults with the nt decode streams
set -o pipefail
mkdir -p gpurun_out
LLMD_MOE_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_moe_llama.py \
  -k "moe" > gpurun_out/r4ab_tests.log 2>&1 || { tail -30 gpurun_out/r4ab_tests.log; exit 1; }
tail -1 gpurun_out/r4ab_tests.log
for cfg in "fp8 256 0" "fp8 256 1" "fp8 256 0" "fp8 256 1" "bf16 112 0" "bf16 112 1"; do
  set -- $cfg
  Q=""; [ $1 = fp8 ] && Q="--quantization fp8"
  LLMD_MOE_NT=$3 timeout -k 10 400 python -u scripts/bench_decode.py --model gpt-oss-120b --batch $2 --isl 5150 --steps 60 $Q \
    > gpurun_out/r4ab_$1_$3.log 2>&1 || { tail -20 gpurun_out/r4ab_$1_$3.log; exit 1; }
  echo "$1 batch $2 MOE_NT=$3: $(grep 'decode batch' gpurun_out/r4ab_$1_$3.log)" | tee -a gpurun_out/r4ab_summary.txt
done
timeout -k 10 600 python bench.py > gpurun_out/r4ab_bench.out 2> gpurun_out/r4ab_bench.err || { tail -20 gpurun_out/r4ab_bench.err; exit 1; }
grep "timed step" gpurun_out/r4ab_bench.err | tail -1; tail -1 gpurun_out/r4ab_bench.out | cut -c1-300
