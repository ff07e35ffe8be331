# Llama-3-70B decode-only steps (batch 64, ctx 5000, hipGraphs) on one GPU: step time + last-window kernel breakdown.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_d70r5 -o run -- python3 scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 40 > gpurun_out/d70r5_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/d70r5_bench.log; exit 1; }
f=$(find /tmp/prof_d70r5 -name '*kernel_trace.csv' | head -1)
{ grep "decode batch" gpurun_out/d70r5_bench.log; python scripts/busy_from_trace.py "$f" 1.0 --breakdown; } | tee gpurun_out/d70r5_summary.txt
rm -f "$f"
