# Round-2 regression: all GPU tests, smoke, driver-shaped 1-GPU bench, 4- and 8-rank P/D rehearsals.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${GPU_TESTS_FROM:-} > gpurun_out/gpu_all.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_n1.log; exit 1; }
grep '^{' gpurun_out/bench_n1.log | cut -c1-300
bash scripts/gpu_pd.sh && bash scripts/gpu_pd8.sh
