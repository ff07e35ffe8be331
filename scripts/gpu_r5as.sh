# Kernel breakdown of the gpt-oss-120b block-fp8 serving bench (256 in flight, ISL 5150): where the 90 ms prefill
# steps go beyond the MoE GEMMs.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 20 --warmup 5 --quantization fp8 --concurrency 256"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_r5as -o run -- python3 bench.py $M > gpurun_out/r5as_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5as_bench.log; exit 1; }
f=$(find /tmp/prof_r5as -name '*kernel_trace.csv' | head -1)
{ grep -E "timed step sizes" gpurun_out/r5as_bench.log; python3 scripts/busy_from_trace.py "$f" 3.0 --breakdown; } | tee gpurun_out/r5as_summary.txt
rm -f "$f"
