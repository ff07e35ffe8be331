# gpt-oss-120b (the reference's published P/D model) aggregated on one MI355X:
# bench at two concurrencies + a kernel-trace breakdown of the timed window.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
M="--model gpt-oss-120b --isl 5150 --osl 250"
timeout -k 10 400 python bench.py $M --concurrency 112 --steps 40 --warmup 10 > gpurun_out/gptoss_c112.log 2>&1 || { echo "c112 failed"; tail -20 gpurun_out/gptoss_c112.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gptoss_c112.log | cut -c1-400
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gptoss -o run -- python3 bench.py $M --concurrency 64 --steps 40 --warmup 10 > gpurun_out/gptoss_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/gptoss_prof.log; exit 1; }
f=$(find gpurun_out/prof_gptoss -name '*kernel_trace.csv' | head -1)
{ python scripts/busy_from_trace.py "$f" 2.5; python scripts/busy_from_trace.py "$f" 2.5 --breakdown; } > gpurun_out/gptoss_busy.txt
rm -f "$f"
head -30 gpurun_out/gptoss_busy.txt
timeout -k 10 300 python bench.py --steps 40 --warmup 10 > gpurun_out/b70_steps.log 2>&1 || { echo "70b failed"; tail -20 gpurun_out/b70_steps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b70_steps.log | cut -c1-400
