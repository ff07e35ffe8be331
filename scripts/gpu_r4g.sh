# round 4 (g): PMC of the MLA v2 rows-64 decode (shape 41), then the bench with and
# without LLMD_ALIGN_KEEP_FINAL over 60 steps
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export LLMD_MLA_SHAPE=41
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_mla41_a -- python3 $R/scripts/bench_attn.py --mla-only --rows 64 > $R/gpurun_out/pmc_mla41_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mla41_b -- python3 $R/scripts/bench_attn.py --mla-only --rows 64 > $R/gpurun_out/pmc_mla41_b.log 2>&1 || exit $?
echo pmc done
unset LLMD_MLA_SHAPE
cd $R
for kf in 0 1; do
  LLMD_ALIGN_KEEP_FINAL=$kf timeout -k 10 600 python -u bench.py --steps 60 --warmup 5 > gpurun_out/bench60_kf$kf.out 2> gpurun_out/bench60_kf$kf.err || exit $?
  grep "timed step" gpurun_out/bench60_kf$kf.err | tail -1
  tail -1 gpurun_out/bench60_kf$kf.out | cut -c1-260
done
