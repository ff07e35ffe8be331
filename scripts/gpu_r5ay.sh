# (pending: apply docs/pending/decode_graph_single_copy.patch first) Decode graph inputs through one pinned mirror + one H2D copy: the engine/graph GPU tests, then the driver bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_models_gpu.py tests/test_shared_prefix_gpu.py tests/test_fp8_kv.py tests/test_hybrid_kv.py \
  tests/test_mgemm.py tests/test_engine.py tests/test_ep_gpu.py > gpurun_out/r5ay_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5ay_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ay_bench.log 2>&1
rc=$?; grep -E "timed step sizes" gpurun_out/r5ay_bench.log; grep '^{' gpurun_out/r5ay_bench.log | cut -c1-200; exit $rc
