# round 4 (f): MLA kernel shapes (41 = v2 two 64-head workgroups, 81 = v2 8 waves,
# 42 = v3 32 heads per wave) timed, v3 numerics, PMC of the rows-64 decode for
# 41 and 42, then the bench with and without LLMD_ALIGN_KEEP_FINAL over 60 steps
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for sh in 41 81 42; do
  LLMD_MLA_SHAPE=$sh timeout -k 10 150 python -u scripts/bench_attn.py --mla-only > gpurun_out/mla_shape_$sh.log 2>&1 || exit $?
  grep "^mla" gpurun_out/mla_shape_$sh.log | sed "s/^/shape $sh: /"
done
LLMD_MLA_SHAPE=42 timeout -k 10 300 python -u -m pytest tests/test_deepseek.py tests/test_fp8_kv.py -k mla -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/mla42_tests.log 2>&1
rc=$?
tail -3 gpurun_out/mla42_tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for sh in 41 42; do
  export LLMD_MLA_SHAPE=$sh
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_mla${sh}_a -- python3 $R/scripts/bench_attn.py --mla-only --rows 64 > $R/gpurun_out/pmc_mla${sh}_a.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mla${sh}_b -- python3 $R/scripts/bench_attn.py --mla-only --rows 64 > $R/gpurun_out/pmc_mla${sh}_b.log 2>&1 || exit $?
done
unset LLMD_MLA_SHAPE
cd $R
for kf in 0 1; do
  LLMD_ALIGN_KEEP_FINAL=$kf timeout -k 10 600 python -u bench.py --steps 60 --warmup 5 > gpurun_out/bench60_kf$kf.out 2> gpurun_out/bench60_kf$kf.err || exit $?
  grep "timed step" gpurun_out/bench60_kf$kf.err | tail -1
  tail -1 gpurun_out/bench60_kf$kf.out | cut -c1-260
done
