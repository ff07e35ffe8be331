# round 4 (u): bench with the 518 -> 512 trim, twice (defaults), engine GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_engine.py -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4u_t.log 2>&1 || { tail -5 gpurun_out/r4u_t.log; exit 1; }
tail -1 gpurun_out/r4u_t.log
for i in 1 2; do
  timeout -k 10 900 python -u bench.py > gpurun_out/r4u_bench$i.out 2> gpurun_out/r4u_bench$i.err || { tail -20 gpurun_out/r4u_bench$i.err; exit 1; }
  grep "timed step" gpurun_out/r4u_bench$i.err | tail -1
  tail -1 gpurun_out/r4u_bench$i.out | cut -c1-240
done
