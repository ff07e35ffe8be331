# kernel split of the default bf16 70B serving bench's timed window (rocprofv3 kernel trace, last 3.3 s = 20 steps)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 rocprofv3 --kernel-trace -d gpurun_out/r6s_prof -o run -- python3 bench.py --steps 20 --warmup 5 --fp8-extra off > gpurun_out/r6s.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r6s.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 gpurun_out/r6s.log; exit $rc; }
f=$(find gpurun_out/r6s_prof -name "*kernel_trace.csv" -o -name "*results.db" | head -1)
python3 scripts/kernel_window.py "$f" 3.3 30 > gpurun_out/r6s_window.txt && cat gpurun_out/r6s_window.txt
rm -f "$f"
