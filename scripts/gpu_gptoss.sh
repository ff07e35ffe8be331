# gpt-oss-120b (the reference's published P/D model) aggregated on one MI355X:
# padded-K fp8 MoE numerics, benches (bf16 / block-fp8 experts) and a kernel-trace breakdown.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 || { echo "fp8 tests failed"; tail -30 gpurun_out/fp8_tests.log; exit 1; }
tail -1 gpurun_out/fp8_tests.log
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10"
for c in 64 128; do
  timeout -k 10 400 python bench.py $M --quantization fp8 --concurrency $c > gpurun_out/gptoss_fp8_c$c.log 2>&1 || { echo "fp8 c$c failed"; tail -20 gpurun_out/gptoss_fp8_c$c.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/gptoss_fp8_c$c.log | cut -c1-330
done
timeout -k 10 400 python bench.py $M --concurrency 112 > gpurun_out/gptoss_c112.log 2>&1 || { echo "c112 failed"; tail -20 gpurun_out/gptoss_c112.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gptoss_c112.log | cut -c1-330
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gptoss -o run -- python3 bench.py $M --quantization fp8 --concurrency 128 > gpurun_out/gptoss_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/gptoss_prof.log; exit 1; }
f=$(find gpurun_out/prof_gptoss -name '*kernel_trace.csv' | head -1)
{ python scripts/busy_from_trace.py "$f" 2.5; python scripts/busy_from_trace.py "$f" 2.5 --breakdown; } > gpurun_out/gptoss_busy.txt
rm -f "$f"
head -30 gpurun_out/gptoss_busy.txt
timeout -k 10 300 python bench.py --steps 40 --warmup 10 > gpurun_out/b70_steps.log 2>&1 || { echo "70b failed"; tail -20 gpurun_out/b70_steps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b70_steps.log | cut -c1-330
