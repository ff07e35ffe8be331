set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_shared_prefix_gpu.py tests/test_models_gpu.py -x -q -k "paged_decode or shared_prefix or splits or gpu" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/nsplit_test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/nsplit_test.log; exit 1; }
tail -1 gpurun_out/nsplit_test.log
timeout -k 10 200 python -u scripts/bench_decode_nsplit.py 2>&1 | grep -v amdgpu.ids > gpurun_out/decode_nsplit.log || exit 1
cat gpurun_out/decode_nsplit.log
bash scripts/gpu_ob_ladder2.sh
