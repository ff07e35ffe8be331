# (1) 2-rank aggregated (dp2) rehearsal of bench.py on one GPU (small model, gloo control);
# (2) rocprofv3 kernel trace + stats of the 1-GPU 70B bench at the driver's default step counts.
set -o pipefail
mkdir -p gpurun_out
LLMD_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 20 --warmup 5 --model llama-3-8b \
  --kv-cache-gb 20 --concurrency 16 > gpurun_out/agg2_rehearsal.log 2>&1 || { echo "agg2 failed"; tail -30 gpurun_out/agg2_rehearsal.log; exit 1; }
grep '^{' gpurun_out/agg2_rehearsal.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_n1
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_n1 -o run -- python3 bench.py --steps 40 --warmup 20 > gpurun_out/prof_n1_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_n1_bench.log; exit 1; }
f=$(find gpurun_out/prof_n1 -name '*kernel_trace.csv' | head -1)
python3 scripts/busy_from_trace.py "$f" 6.5 --breakdown > gpurun_out/prof_n1_summary.txt
s=$(find gpurun_out/prof_n1 -name '*kernel_stats.csv' | head -1)
cp "$s" gpurun_out/prof_n1_kernel_stats.csv
rm -f "$f"
grep '^{' gpurun_out/prof_n1_bench.log | cut -c1-300
cut -c1-160 gpurun_out/prof_n1_summary.txt | head -25
