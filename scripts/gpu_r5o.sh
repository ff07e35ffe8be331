# prefill attention v4 with the asm LDS-DMA (counted lgkmcnt waits): numerics + 3-arm A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_prefill_v4.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5o_attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5o_attn_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/attn_v4_ab.py > gpurun_out/r5o_attn_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5o_attn_ab.log | grep "AB\|check"; exit $rc
