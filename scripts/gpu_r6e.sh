# Round 6: async scheduling on the GPU - full GPU suite, 70B decode step on/off, bench.py, gpt-oss on/off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6e_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6e_gpu_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r6e_gpu_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
for m in on off; do
  x=""; [ $m = off ] && x="--no-async-scheduling"
  timeout -k 10 400 python -u scripts/bench_decode.py --steps 60 $x > gpurun_out/r6e_decode_$m.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r6e_decode_$m.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --fp8-extra off > gpurun_out/r6e_bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6e_bench.log | tail -3; [ $rc -eq 0 ] || exit $rc
for m in on off; do
  x=""; [ $m = off ] && x="--no-async-scheduling"
  timeout -k 10 500 python -u bench.py --model gpt-oss-120b --isl 5150 --osl 250 --quantization fp8 --concurrency 256 --steps 60 --warmup 5 $x > gpurun_out/r6e_gptoss_$m.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r6e_gptoss_$m.log | grep -E "timed|^\{" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
