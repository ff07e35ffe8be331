# End-to-end serving on one MI355X: 2 Llama-3-8B replicas (one process each, same GPU) behind the router,
# shared-prefix load through HTTP under three routing policies (scripts/e2e_serving.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/e2e_serving.py --model llama-3-8b --device cuda --replicas 2 --blocks 4096 \
  --groups 48 --per-group 16 --system-len 2048 --question-len 128 --output-len 64 --concurrency 64 --requests 768 --configs prefix,precise,load,random,prefix,precise \
  --out gpurun_out/e2e_serving.json > gpurun_out/e2e_serving.log 2>&1
rc=$?
grep "^\[e2e\]" gpurun_out/e2e_serving.log | grep -v "\.\.\." | cut -c1-400
[ $rc -eq 0 ] || { tail -30 gpurun_out/e2e_serving.log; tail -20 gpurun_out/e2e_engine0.log; }
exit $rc
