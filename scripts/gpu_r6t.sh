# prefill attention default V53: numerics (every prefill GPU test), then the bf16 bench kernel window
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu -k "prefill" > gpurun_out/r6t_test.log 2>&1 || { tail -30 gpurun_out/r6t_test.log; exit 1; }
tail -2 gpurun_out/r6t_test.log
bash scripts/gpu_r6s.sh
