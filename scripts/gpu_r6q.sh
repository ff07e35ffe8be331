# full GPU suite + smoke + default bench (round-6 validation after the persistent MoE GEMMs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6q_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r6q_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6q_smoke.log 2>&1 || { tail -20 gpurun_out/r6q_smoke.log; exit 1; }
tail -2 gpurun_out/r6q_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r6q_bench.log 2>&1; rc=$?
grep '"metric"' gpurun_out/r6q_bench.log | cut -c1-600; exit $rc
