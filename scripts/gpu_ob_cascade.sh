# optimized-baseline shape on one MI355X (Qwen3-32B bf16 replica behind the router, shared-prefix load,
# 19 prefix groups of 6000 tokens + 1200-token questions, 360 output tokens): shared-prefix decode on vs off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shared_prefix_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cascade_engine_test.log 2>&1 || { echo "engine test failed"; tail -30 gpurun_out/cascade_engine_test.log; exit 1; }
tail -1 gpurun_out/cascade_engine_test.log
for mode in on off; do
  extra="--extra-engine-args="
  [ $mode = off ] && extra="--extra-engine-args=--disable-shared-prefix-decode"
  timeout -k 10 600 python -u scripts/e2e_serving.py --model qwen3-32b --device cuda --replicas 1 --blocks 40000 \
    --configs prefix --system-len 6000 --question-len 1200 --output-len 360 \
    --workload guide_optimized-baseline_1.yaml "$extra" --concurrency 160 \
    --overrides "load.stages=[{rate: 4, duration: 40}, {rate: 6, duration: 40}, {rate: 8, duration: 40}],data.shared_prefix.num_groups=19" \
    --out gpurun_out/ob_cascade_$mode.json > gpurun_out/ob_cascade_$mode.log 2>&1
  rc=$?
  echo "== shared-prefix decode $mode"
  grep "^\[e2e\]" gpurun_out/ob_cascade_$mode.log | grep -v "\.\.\." | cut -c1-330
  [ $rc -eq 0 ] || { tail -30 gpurun_out/ob_cascade_$mode.log; tail -20 gpurun_out/e2e_engine0.log; exit $rc; }
done
