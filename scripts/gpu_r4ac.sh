# round 4 (ac): final validation with the nt decode-stream defaults - full GPU suite, smoke(), then gpt-oss-120b
# fp8 c256 / bf16 c112 at ISL 5150 (the README table rows)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4ac_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4ac_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r4ac_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ac_smoke.log 2>&1 || { tail -20 gpurun_out/r4ac_smoke.log; exit 1; }
tail -1 gpurun_out/r4ac_smoke.log
M="--model gpt-oss-120b --isl 5150 --osl 250 --steps 40 --warmup 10"
timeout -k 10 500 python bench.py $M --quantization fp8 --concurrency 256 > gpurun_out/r4ac_fp8_c256.out 2> gpurun_out/r4ac_fp8_c256.err || { tail -20 gpurun_out/r4ac_fp8_c256.err; exit 1; }
grep "timed step" gpurun_out/r4ac_fp8_c256.err | tail -1; tail -1 gpurun_out/r4ac_fp8_c256.out | cut -c1-200
timeout -k 10 500 python bench.py $M --concurrency 112 > gpurun_out/r4ac_bf16_c112.out 2> gpurun_out/r4ac_bf16_c112.err || { tail -20 gpurun_out/r4ac_bf16_c112.err; exit 1; }
grep "timed step" gpurun_out/r4ac_bf16_c112.err | tail -1; tail -1 gpurun_out/r4ac_bf16_c112.out | cut -c1-200
