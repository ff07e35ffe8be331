# gpt-oss-120b fp8 serving, steady-state window: MoE fp8 v4 (threshold 96, r6 start) vs v8 + threshold 56
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --model gpt-oss-120b --isl 5150 --osl 250 --quantization fp8 --concurrency 256 --steps 60 --warmup 5 --fp8-extra off > gpurun_out/r6o_$n.log 2>&1 || { tail -20 gpurun_out/r6o_$n.log; return 1; }
  echo "== $n"; grep '"metric"' gpurun_out/r6o_$n.log
}
run v4 LLMD_MOE_FP8_V8=0 LLMD_MOE_V3_MIN_ROWS=96 && run v8 LLMD_MOE_FP8_V8=1
