# kernel split of gpt-oss-120b fp8 serving's timed window (256 in flight, ISL 5150 / OSL 250, 20 steps)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 800 rocprofv3 --kernel-trace -d gpurun_out/r6aa_prof -o run -- python3 bench.py --model gpt-oss-120b --isl 5150 --osl 250 --quantization fp8 --concurrency 256 --steps 20 --warmup 5 --fp8-extra off > gpurun_out/r6aa.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r6aa.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 gpurun_out/r6aa.log; exit $rc; }
f=$(find gpurun_out/r6aa_prof -name "*results.db" -o -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_window.py "$f" 1.6 30 > gpurun_out/r6aa_window.txt && cat gpurun_out/r6aa_window.txt
rm -f "$f"
