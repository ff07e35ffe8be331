# round 4 (q): kernel breakdown of the driver's bench with the final round-4 code (stats only; the trace stays in /tmp)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/r4q_bench.out 2> $R/gpurun_out/r4q_bench.err
rc=$?
mkdir -p $R/gpurun_out/prof_bench && cp /tmp/prof_bench/*/*kernel_stats.csv $R/gpurun_out/prof_bench/ 2>/dev/null
grep "timed step" $R/gpurun_out/r4q_bench.err | tail -1
tail -1 $R/gpurun_out/r4q_bench.out | cut -c1-200
exit $rc
