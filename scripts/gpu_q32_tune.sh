# prefill v2 on 16-key blocks (numerics), then TunableOp for the Qwen3-32B mixed-step GEMM shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "prefill" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/prefill_bs16_test.log 2>&1 || { echo "prefill tests failed"; tail -40 gpurun_out/prefill_bs16_test.log; exit 1; }
tail -1 gpurun_out/prefill_bs16_test.log
timeout -k 10 200 python -u scripts/bench_attn.py --help > /dev/null 2>&1
timeout -k 10 900 python -u scripts/tune_gemm.py --models qwen3-32b --ms 512 1024 --names qkv o gate_up down --out gpurun_out/tunableop_q32.csv > gpurun_out/tune_q32.log 2>&1
rc=$?
tail -12 gpurun_out/tune_q32.log
exit $rc
