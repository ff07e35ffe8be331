# Round 6: steady-state bench windows (tools/steady.py) for 70B / 8B / gpt-oss at the
# driver's arguments and over 250 steps, plus the symm "later barriers give up" test.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_collective_failure.py > gpurun_out/r6a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6a_tests.log; [ $rc -eq 0 ] || exit $rc
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
