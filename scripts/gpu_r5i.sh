# BASELINE config 5 re-measured: the round-3 load (scripts/gpu_e2e_tiered_gptoss.sh) on one
# gpt-oss-120b replica with the hybrid KV manager (default for windowed models) and the async tier reload.
#   A: the same 8192 full-attention blocks (131k tokens of context) as round 3, host tier 0 / 60 GB;
#   B: the same KV BYTES as round 3's 8192 blocks x 36 layers (9663676416 B): the hybrid manager turns them into
#      ~2x the full-attention blocks (18 full layers; the windowed pool is small), host tier 0 / 60 GB.
set -o pipefail
mkdir -p gpurun_out
common="--model gpt-oss-120b --device cuda --replicas 1 --groups 64 --per-group 8 --system-len 4096
  --question-len 256 --output-len 128 --concurrency 64 --requests 512 --configs random"
for run in A B; do
  for tier in 0 60; do
    if [ $run = A ]; then sz="--blocks 8192"; xa="--quantization fp8"; else sz="--blocks 0"; xa="--quantization fp8 --kv-cache-memory-bytes 9663676416"; fi
    timeout -k 10 600 python -u scripts/e2e_serving.py $common $sz --kv-offload-gb $tier --extra-engine-args="$xa" \
      --out gpurun_out/r5i_${run}_$tier.json > gpurun_out/r5i_${run}_$tier.log 2>&1 \
      || { tail -30 gpurun_out/r5i_${run}_$tier.log; tail -20 gpurun_out/e2e_engine0.log; exit 1; }
    echo "== run ${run} host tier ${tier} GB"
    grep -h "hybrid KV cache\|kv cache:" gpurun_out/e2e_engine0.log | head -2 | cut -c1-200
    grep "^\[e2e\] random" gpurun_out/r5i_${run}_$tier.log | cut -c1-420
  done
done
