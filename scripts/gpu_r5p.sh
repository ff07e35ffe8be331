# P/D same-device checks; MoE v4 192-row tiles numerics; the driver bench with / without the mixed-step
# attention overlap; MoE A/B; prefill attention 4-arm A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pd_cross_device.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5p_pd.log 2>&1
rc=$?; tail -2 gpurun_out/r5p_pd.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_kv.py -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "moe" > gpurun_out/r5p_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5p_tests.log; [ $rc -ne 0 ] && exit $rc
for ov in 1 0; do
  LLMD_ATTN_OVERLAP=$ov timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5p_bench_$ov.out 2> gpurun_out/r5p_bench_$ov.err
  rc=$?; echo "overlap=$ov: $(grep 'timed step' gpurun_out/r5p_bench_$ov.err) $(grep -o '"value": [0-9.]*' gpurun_out/r5p_bench_$ov.out)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r5p_bench_$ov.err; exit $rc; }
done
timeout -k 10 600 python -u scripts/bench_moe.py > gpurun_out/r5p_moe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5p_moe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_prefill_v4.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5p_attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5p_attn_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/attn_v4_ab.py > gpurun_out/r5p_attn_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5p_attn_ab.log | grep "AB\|check"; exit $rc
