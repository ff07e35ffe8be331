set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_shared_prefix_gpu.py -x -q -k "paged_decode or shared_prefix or splits" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/split_dev_test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/split_dev_test.log; exit 1; }
tail -1 gpurun_out/split_dev_test.log
timeout -k 10 200 python -u scripts/bench_decode_split.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/decode_split.log
