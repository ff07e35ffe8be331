# BASELINE config 2 (Llama-3-8B optimized-baseline, prefix-cache-aware routing) on one MI355X: two Llama-3-8B
# replicas (one process each, same GPU) behind the router with the guide's EPP config, guide_optimized-baseline_1
# load (shared 6000-token prefixes + 1200-token questions, 360 output tokens), 38 prefix groups, rate ladder
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/e2e_serving.py --model llama-3-8b --device cuda --replicas 2 --blocks 30000 \
  --configs prefix --system-len 6000 --question-len 1200 --output-len 360 \
  --workload guide_optimized-baseline_1.yaml --concurrency 192 \
  --overrides "load.stages=[{rate: 8, duration: 40}, {rate: 16, duration: 40}, {rate: 24, duration: 40}, {rate: 32, duration: 40}, {rate: 40, duration: 40}],data.shared_prefix.num_groups=38" \
  --out gpurun_out/ob_8b.json > gpurun_out/ob_8b.log 2>&1
rc=$?
grep "^\[e2e\]" gpurun_out/ob_8b.log | grep -v "\.\.\." | cut -c1-330
[ $rc -eq 0 ] || { tail -30 gpurun_out/ob_8b.log; tail -20 gpurun_out/e2e_engine0.log; }
exit $rc
