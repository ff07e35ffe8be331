# Round 6: steady-state bench windows (tools/steady.py) for 70B / 8B / gpt-oss at the
# driver's arguments and over 250 steps, (the symm stall test runs in gpu_r6b.sh).
set -o pipefail
mkdir -p gpurun_out
run() {  # name, timeout, args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > gpurun_out/r6a_$n.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r6a_$n.log | tail -4; [ $rc -eq 0 ] || exit $rc
}
run 70b_k20 400 --gpus 1 --steps 20 --warmup 5
run 70b_k250 500 --gpus 1 --steps 250 --warmup 5
run 8b_k20 400 --model llama-3-8b --concurrency 256 --steps 20 --warmup 5
run 8b_k250 400 --model llama-3-8b --concurrency 256 --steps 250 --warmup 5
run gptoss_k20 400 --model gpt-oss-120b --isl 5150 --osl 250 --quantization fp8 --concurrency 256 --steps 20 --warmup 5
run gptoss_k250 500 --model gpt-oss-120b --isl 5150 --osl 250 --quantization fp8 --concurrency 256 --steps 250 --warmup 5
