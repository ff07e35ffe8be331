# optimized-baseline guide workload on one MI355X: one Qwen3-32B bf16 replica (the reference runs 8 replicas
# of TP2 on 16 H100) behind the router with the guide's EPP config, shared-prefix load ladder at the
# reference's per-replica rates (its 3..60 req/s ladder / 8 replicas), 1/8 of the prefix groups.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/e2e_serving.py --model qwen3-32b --device cuda --replicas 1 --blocks 40000 \
  --configs prefix --system-len 6000 --question-len 1200 --output-len 360 \
  --workload guide_optimized-baseline_1.yaml \
  --overrides "load.stages=[{rate: 1, duration: 40}, {rate: 2, duration: 40}, {rate: 3, duration: 40}, {rate: 4, duration: 40}, {rate: 5, duration: 40}, {rate: 6, duration: 40}, {rate: 7.5, duration: 40}],data.shared_prefix.num_groups=19" \
  --out gpurun_out/optbaseline_32b.json > gpurun_out/optbaseline_32b.log 2>&1
rc=$?
grep "^\[e2e\]" gpurun_out/optbaseline_32b.log | grep -v "\.\.\." | cut -c1-330
[ $rc -eq 0 ] || { tail -30 gpurun_out/optbaseline_32b.log; tail -20 gpurun_out/e2e_engine0.log; }
exit $rc
