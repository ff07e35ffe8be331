# round 4 (i): numerics after the asm LDS-DMA change (prefill v2, MLA v2/v3), MLA split sweep
# with the v3 default, kernel-level MLA breakdown, GQA prefill/decode timing
set -o pipefail
mkdir -p gpurun_out
# the round-4 kernels under test (opt-in until these numerics pass)
export LLMD_PREFILL_V3=1 LLMD_MOE_V3_BF16=1
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_deepseek.py tests/test_kernels_prod_shapes.py tests/test_shared_prefix_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4i_tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" gpurun_out/r4i_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u scripts/bench_mla_split.py > gpurun_out/mla_split_v3.log 2>&1 || exit $?
grep rows gpurun_out/mla_split_v3.log
LLMD_MLA_PARTIAL_BF16=1 timeout -k 10 200 python -u -m pytest tests/test_deepseek.py -q -x -k mla_kernel --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/mla_pbf16_test.log 2>&1 || { tail -5 gpurun_out/mla_pbf16_test.log; exit 1; }
LLMD_MLA_PARTIAL_BF16=1 timeout -k 10 150 python -u scripts/bench_attn.py --mla-only > gpurun_out/mla_pbf16.log 2>&1 || exit $?
grep "^mla" gpurun_out/mla_pbf16.log | sed "s/^/partial bf16: /"
timeout -k 10 150 python -u scripts/bench_attn.py --mla-only > gpurun_out/mla_pf32.log 2>&1 || exit $?
grep "^mla" gpurun_out/mla_pf32.log | sed "s/^/partial f32: /"
timeout -k 10 200 python -u scripts/bench_attn.py --check > gpurun_out/attn_r4i.log 2>&1 || exit $?
grep -E "^(prefill|decode|  prefill check)" gpurun_out/attn_r4i.log
LLMD_PREFILL_V3=0 timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/attn_r4i_v2.log 2>&1 || exit $?
grep -E "^prefill" gpurun_out/attn_r4i_v2.log | sed "s/^/v2: /"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mla_v3 -- python3 $R/scripts/bench_attn.py --mla-only --rows 64 > $R/gpurun_out/prof_mla_v3.log 2>&1 || exit $?
echo prof done
cd $R
timeout -k 10 400 python -u -m pytest tests/test_fp8_kv.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "moe" -p no:cacheprovider > gpurun_out/moe_r4i_tests.log 2>&1 || { echo "moe tests failed"; grep -E "^E |FAILED" gpurun_out/moe_r4i_tests.log | head; exit 1; }
tail -1 gpurun_out/moe_r4i_tests.log
timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/moe_r4i_bench.txt 2>&1 || { echo bench failed; tail -20 gpurun_out/moe_r4i_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/moe_r4i_bench.txt
LLMD_MOE_V3_BF16=0 timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/moe_r4i_bench_v2bf16.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/moe_r4i_bench_v2bf16.txt | sed "s/^/bf16 v2: /"
timeout -k 10 200 python -u scripts/bench_shared_prefix.py > gpurun_out/shared_prefix_r4i.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/shared_prefix_r4i.txt | tail -12
