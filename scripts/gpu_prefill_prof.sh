# Kernel breakdown of a P/D prefill rank (70B, ISL 5000 prompts, max_tokens=1, 8192-token chunks).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_pre
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_pre -o run -- python3 scripts/bench_prefill_rate.py --steps 12 > gpurun_out/prefill_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prefill_prof.log; exit 1; }
f=$(find gpurun_out/prof_pre -name '*kernel_trace.csv' | head -1)
{ grep "prefill ISL" gpurun_out/prefill_prof.log; python3 scripts/busy_from_trace.py "$f" 6.0 --breakdown; } > gpurun_out/prefill_summary.txt
rm -f "$f"
cut -c1-150 gpurun_out/prefill_summary.txt | head -30
