# DeepSeek-V2-Lite decode (MLA + 64-expert MoE, EP=1) on one GPU: step time + last-window kernel breakdown.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dsl -o run -- python3 scripts/bench_decode.py --model deepseek-v2-lite --batch 64 --isl 2000 --steps 60 > gpurun_out/dsl_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/dsl_bench.log; exit 1; }
f=$(find gpurun_out/prof_dsl -name '*kernel_trace.csv' | head -1)
{ grep "decode batch" gpurun_out/dsl_bench.log; python scripts/busy_from_trace.py "$f" 0.5 --breakdown; } | tee gpurun_out/dsl_summary.txt
rm -f "$f"
