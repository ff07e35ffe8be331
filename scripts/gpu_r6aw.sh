# final round-6 validation, part 2: smoke() and the default bench.py
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6aw_smoke.log 2>&1 || { tail -20 gpurun_out/r6aw_smoke.log; exit 1; }
tail -1 gpurun_out/r6aw_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r6aw_bench.log 2>&1; rc=$?
grep '"metric"' gpurun_out/r6aw_bench.log | cut -c1-400; exit $rc
