# round 4 (b): production-shape attention numerics, then the one-EP-rank DeepSeek-R1
# projection (fp8 dispatch kernels in loopback + the 61-layer decode step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_prod_shapes.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b_prod_shapes.log 2>&1
rc=$?
tail -4 gpurun_out/r4b_prod_shapes.log
[ $rc -ne 0 ] && { grep -E "Error|error|FAILED|assert|Mismatch" gpurun_out/r4b_prod_shapes.log | head -30; exit $rc; }
timeout -k 10 200 python -u scripts/bench_attn.py --mla --ctx 4096 > gpurun_out/mla_pair.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/mla_pair.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_ep_recv.py > gpurun_out/ep_recv.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/ep_recv.log | tail -4
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/bench_wide_ep_rank.py --steps 20 --out gpurun_out/wide_ep_rank_r1.json > gpurun_out/wide_ep_rank.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/wide_ep_rank.log | tail -12
[ $rc -ne 0 ] && exit $rc
# kernel-level breakdown of the one-rank decode step (MLA, grouped GEMMs, symm dispatch/combine);
# the full trace stays in /tmp (it exceeds gpurun_out's 64 MiB), only the stats are copied back
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_wide_ep_rank -- python3 $R/scripts/bench_wide_ep_rank.py --steps 5 --out /tmp/wide_ep_rank_prof.json > $R/gpurun_out/prof_wide_ep_rank.log 2>&1
rc=$?
echo "prof rc=$rc"
mkdir -p $R/gpurun_out/prof_wide_ep_rank && cp /tmp/prof_wide_ep_rank/*/*kernel_stats.csv $R/gpurun_out/prof_wide_ep_rank/ 2>/dev/null
exit $rc
