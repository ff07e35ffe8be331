# bf16 + block-fp8 MoE v4 numerics + A/B vs v3 and fp8 (DeepSeek EP8 / gpt-oss shapes), then the gpt-oss-120b KV capacity
# with and without the hybrid manager at a fixed --gpu-memory-utilization
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "moe_experts" > gpurun_out/r5h_tests.log 2>&1 && timeout -k 10 300 python -u -m pytest tests/test_fp8_kv.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "moe" >> gpurun_out/r5h_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5h_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/bench_moe.py > gpurun_out/r5h_moe.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5h_moe.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/kv_capacity.py --model gpt-oss-120b --quantization fp8 > gpurun_out/r5h_capacity.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r5h_capacity.log | tail -4
exit $rc
