# MoE v4 with the 192-row tiles fixed: A/B (scripts/bench_moe.py), P/D same-device checks, gpt-oss-120b fp8 at 256 in
# flight with auto tiles vs forced 256-row tiles, then the 70B driver bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_moe.py > gpurun_out/r5s_moe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5s_moe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_pd_cross_device.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5s_pd.log 2>&1
rc=$?; tail -2 gpurun_out/r5s_pd.log; [ $rc -ne 0 ] && exit $rc
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10 --quantization fp8 --concurrency 256"
for t in auto 256; do
  LLMD_MOE4_TILE=$t timeout -k 10 500 python bench.py $M > gpurun_out/r5s_gptoss_$t.log 2>&1
  rc=$?; echo "tile=$t: $(grep -v amdgpu.ids gpurun_out/r5s_gptoss_$t.log | grep '^{' | cut -c1-260)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r5s_gptoss_$t.log; exit $rc; }
done
exit 0
