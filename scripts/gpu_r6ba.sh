# final round-6 validation, part 1: the full GPU suite (final tree)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6ba_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r6ba_gpu.log
exit $rc
