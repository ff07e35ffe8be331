# BASELINE config 5 (gpt-oss-120b + tiered KV prefix cache offload to host DRAM) on one MI355X: one gpt-oss-120b
# replica (fp8 experts) whose HBM KV pool (8192 x 16-token blocks = 131k tokens) holds about half of the
# workload's shared prefixes (64 groups x 4096 tokens), with and without a 60 GB host-DRAM tier.
set -o pipefail
mkdir -p gpurun_out
common="--model gpt-oss-120b --device cuda --replicas 1 --blocks 8192 --groups 64 --per-group 8 --system-len 4096
  --question-len 256 --output-len 128 --concurrency 64 --requests 512 --configs random"
for tier in 0 60; do
  timeout -k 10 600 python -u scripts/e2e_serving.py $common --kv-offload-gb $tier --extra-engine-args="--quantization fp8" \
    --out gpurun_out/e2e_tiered_gptoss_$tier.json > gpurun_out/e2e_tiered_gptoss_$tier.log 2>&1 \
    || { tail -30 gpurun_out/e2e_tiered_gptoss_$tier.log; tail -20 gpurun_out/e2e_engine0.log; exit 1; }
  echo "== host tier ${tier} GB"
  grep "^\[e2e\] random" gpurun_out/e2e_tiered_gptoss_$tier.log | cut -c1-420
done
