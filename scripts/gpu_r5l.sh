# Decode A/B after the fixup fence change (release in every split, acquire in the last only) and the fused
# SiLU gate/up mgemm: 70B decode step (batch 64, ctx 5000), then the driver bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mgemm.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5l_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5l_tests.log; [ $rc -ne 0 ] && exit $rc
LLMD_MGEMM_FIXUP=1 timeout -k 10 300 python -u -m pytest tests/test_mgemm.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "split or matches_fp32 or graph" > gpurun_out/r5l_tests_fix.log 2>&1
rc=$?; tail -2 gpurun_out/r5l_tests_fix.log; [ $rc -ne 0 ] && exit $rc
for cfg in "0 0" "0 1" "1 1" "0 1"; do
  set -- $cfg
  LLMD_MGEMM_FIXUP=$1 LLMD_MGEMM_SILU=$2 timeout -k 10 400 python -u scripts/bench_decode.py --steps 40 > gpurun_out/r5l_dec_$1$2.log 2>&1
  rc=$?; echo "fixup=$1 silu=$2: $(grep -v amdgpu.ids gpurun_out/r5l_dec_$1$2.log | tail -1)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5l_bench.out 2> gpurun_out/r5l_bench.err
rc=$?; grep "timed step" gpurun_out/r5l_bench.err; cat gpurun_out/r5l_bench.out; exit $rc
