# Round 6: the routed P/D bench (client -> router/EPP -> decode sidecar -> prefill + kvx) on ONE GPU:
# the 2-process GPU test, then the N=8 topology rehearsal (6P + TP2 decode, then the literal 2P+6D
# with the load-aware decider), llama-3-8b, all ranks on cuda:0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pd_gpu.py > gpurun_out/r6f_pd_test.log 2>&1
rc=$?; tail -3 gpurun_out/r6f_pd_test.log; [ $rc -eq 0 ] || exit $rc
export LLMD_BENCH_DEVICE=0
LLMD_BENCH_STACKS=300 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 30 --warmup 5 --model llama-3-8b \
  --kv-cache-gb 8 --concurrency 16 > gpurun_out/r6f_pd8_rehearsal.log 2>&1
rc=$?; grep -E "routed|router up|^\{" gpurun_out/r6f_pd8_rehearsal.log | cut -c1-1500; [ $rc -eq 0 ] || { tail -30 gpurun_out/r6f_pd8_rehearsal.log; exit $rc; }
