# TP2-shard Llama-3-70B decode (one rank of a TP2 replica) at batch 80 and 128: last-window kernel breakdown.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/dtp_summary.txt
for b in 128; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dtp$b -o run -- python3 scripts/bench_decode.py --model llama-3-70b --tp-shard 2 --batch $b --isl 5000 --steps 30 > gpurun_out/dtp_bench$b.log 2>&1 || { echo "prof $b failed"; tail -20 gpurun_out/dtp_bench$b.log; exit 1; }
  f=$(find gpurun_out/prof_dtp$b -name '*kernel_trace.csv' | head -1)
  { grep "decode batch" gpurun_out/dtp_bench$b.log; python3 scripts/busy_from_trace.py "$f" 0.6 --breakdown; } >> gpurun_out/dtp_summary.txt
  rm -f "$f"
done
cat gpurun_out/dtp_summary.txt | cut -c1-160
