# Tiered prefix cache on one MI355X: one Llama-3-8B replica whose HBM KV pool (65k tokens) holds about a
# third of the workload's shared prefixes (96 groups x 2048 tokens), with and without a 60 GB host-DRAM tier.
set -o pipefail
mkdir -p gpurun_out
common="--model llama-3-8b --device cuda --replicas 1 --blocks 4096 --groups 96 --per-group 8 --system-len 2048
  --question-len 128 --output-len 64 --concurrency 64 --requests 768 --configs random"
timeout -k 10 500 python -u scripts/e2e_serving.py $common --out gpurun_out/e2e_tiered_hbm_only.json \
  > gpurun_out/e2e_tiered_hbm_only.log 2>&1 || { tail -30 gpurun_out/e2e_tiered_hbm_only.log; tail -20 gpurun_out/e2e_engine0.log; exit 1; }
grep "^\[e2e\] random" gpurun_out/e2e_tiered_hbm_only.log | cut -c1-400
timeout -k 10 500 python -u scripts/e2e_serving.py $common --kv-offload-gb 60 --out gpurun_out/e2e_tiered_cpu60.json \
  > gpurun_out/e2e_tiered_cpu60.log 2>&1 || { tail -30 gpurun_out/e2e_tiered_cpu60.log; tail -20 gpurun_out/e2e_engine0.log; exit 1; }
grep "^\[e2e\] random" gpurun_out/e2e_tiered_cpu60.log | cut -c1-400
