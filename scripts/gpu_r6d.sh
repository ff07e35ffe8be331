# Round 6: the driver-style bench with the fp8 extra result; rocprof kernel stats of an fp8 serving run.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6d_bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6d_bench.log | tail -12; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_prof_fp8 -o run -- python3 bench.py --quantization fp8 --kv-cache-dtype fp8 --steps 10 --warmup 2 --fp8-extra off > gpurun_out/r6d_prof.log 2>&1
rc=$?; tail -3 gpurun_out/r6d_prof.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/r6d_prof_fp8 -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -c1-220
