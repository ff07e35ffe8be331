# optimized-baseline shape on one MI355X after prefill v2 on block 16 + Qwen3-32B GEMM tuning (shared-prefix decode on)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/e2e_serving.py --model qwen3-32b --device cuda --replicas 1 --blocks 40000 \
  --configs prefix --system-len 6000 --question-len 1200 --output-len 360 \
  --workload guide_optimized-baseline_1.yaml --concurrency 192 \
  --overrides "load.stages=[{rate: 6, duration: 40}, {rate: 8, duration: 40}, {rate: 10, duration: 40}],data.shared_prefix.num_groups=19" \
  --out gpurun_out/ob_ladder2.json > gpurun_out/ob_ladder2.log 2>&1
rc=$?
grep "^\[e2e\]" gpurun_out/ob_ladder2.log | grep -v "\.\.\." | cut -c1-330
[ $rc -eq 0 ] || { tail -30 gpurun_out/ob_ladder2.log; tail -20 gpurun_out/e2e_engine0.log; }
exit $rc
