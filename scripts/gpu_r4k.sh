# round 4 (k): the full GPU test suite with the defaults, smoke(), then the driver's bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4k_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4k_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r4k_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k_smoke.log 2>&1 || { tail -5 gpurun_out/r4k_smoke.log; exit 1; }
tail -1 gpurun_out/r4k_smoke.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_wide_ep_rank -- python3 $R/scripts/bench_wide_ep_rank.py --steps 5 --out /tmp/wide_ep_rank_prof.json > $R/gpurun_out/prof_wide_ep_rank.log 2>&1
echo "prof rc=$?"
mkdir -p $R/gpurun_out/prof_wide_ep_rank && cp /tmp/prof_wide_ep_rank/*/*kernel_stats.csv $R/gpurun_out/prof_wide_ep_rank/ 2>/dev/null
ls $R/gpurun_out/prof_wide_ep_rank
