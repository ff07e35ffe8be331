set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_busy -o run -- python3 bench.py --steps 30 --warmup 5 > gpurun_out/busy_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/busy_bench.log; exit 1; }
f=$(find gpurun_out/prof_busy -name '*kernel_trace.csv' | head -1)
{ python scripts/busy_from_trace.py "$f" 5.5; python scripts/busy_from_trace.py "$f" 5.5 --breakdown; } | tee gpurun_out/busy_summary.txt
grep '^{' gpurun_out/busy_bench.log | cut -c1-300
rm -f "$f"
