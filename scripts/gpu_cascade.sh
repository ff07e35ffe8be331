# shared-prefix (cascade) decode: numerics vs fp32 reference, then the microbenchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_shared_prefix_gpu.py -x -q -k "paged_decode or shared_prefix" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cascade_test.log 2>&1 || { echo "cascade tests failed"; tail -40 gpurun_out/cascade_test.log; exit 1; }
tail -2 gpurun_out/cascade_test.log
timeout -k 10 200 python -u scripts/bench_shared_prefix.py > gpurun_out/cascade_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/cascade_bench.log; exit 1; }
timeout -k 10 200 python -u scripts/bench_shared_prefix.py --batch 64 --groups 8 --prefix 2048 --suffix 3000 >> gpurun_out/cascade_bench.log 2>&1 || { echo "bench2 failed"; tail -30 gpurun_out/cascade_bench.log; exit 1; }
timeout -k 10 200 python -u scripts/bench_shared_prefix.py --batch 32 --groups 4 --prefix 8192 --suffix 500 >> gpurun_out/cascade_bench.log 2>&1 || { echo "bench3 failed"; tail -30 gpurun_out/cascade_bench.log; exit 1; }
timeout -k 10 200 python -u scripts/bench_shared_prefix.py --bs 16 >> gpurun_out/cascade_bench.log 2>&1 || { echo "bench4 failed"; tail -30 gpurun_out/cascade_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cascade_bench.log
