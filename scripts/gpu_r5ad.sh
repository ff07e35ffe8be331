# Decode reduce fusions (o / down + RMSNorm, QKV + RoPE + cache write): numerics, kernel profile, decode A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_mgemm.py -k "add_rmsnorm or norm_fusion or rope_cache" > gpurun_out/r5ad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5ad_tests.log; [ $rc -ne 0 ] && exit $rc
LLMD_MGEMM_NORM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r5ad -o run -- python3 scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 30 > gpurun_out/r5ad_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r5ad_prof.log; exit 1; }
f=$(find /tmp/prof_r5ad -name '*kernel_trace.csv' | head -1)
python3 scripts/busy_from_trace.py "$f" 1.0 --breakdown | grep -E "reduce|rmsnorm|rope|busy"
for arm in 1 0 1 0; do
  LLMD_MGEMM_NORM=$arm timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 40 > gpurun_out/r5ad_dec$arm.log 2>&1
  rc=$?; echo "norm=$arm $(grep 'decode batch' gpurun_out/r5ad_dec$arm.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r5ad_dec$arm.log; exit $rc; }
done
exit 0
