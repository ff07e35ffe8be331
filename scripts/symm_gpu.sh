set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_symm.py -x -v --timeout 240 --timeout-method thread > gpurun_out/symm_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/symm_tests.log; exit 1; }
echo "symm tests ok"
LLMD_SYMM_BENCH=1 LLMD_SYMM_DEVICE=0 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29655 scripts/symm_check.py > gpurun_out/symm_bench2.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/symm_bench2.log; exit 1; }
tail -2 gpurun_out/symm_bench2.log
