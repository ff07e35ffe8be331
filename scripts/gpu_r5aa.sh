# Decode o / down projections with the residual-add + RMSNorm fused into the split-K reduce
# (ops.mgemm_add_rmsnorm): numerics (bit-identical to the two-kernel path), 70B decode A/B, driver bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_mgemm.py > gpurun_out/r5aa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5aa_tests.log; [ $rc -ne 0 ] && exit $rc
for arm in 1 0 1 0; do
  LLMD_MGEMM_NORM=$arm timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 40 > gpurun_out/r5aa_dec$arm.log 2>&1
  rc=$?; echo "norm=$arm $(grep 'decode batch' gpurun_out/r5aa_dec$arm.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r5aa_dec$arm.log; exit $rc; }
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5aa_bench.log 2>&1
rc=$?; grep -E "timed step sizes" gpurun_out/r5aa_bench.log; grep -o '"value": [0-9.]*' gpurun_out/r5aa_bench.log; exit $rc
