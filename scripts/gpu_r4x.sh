# round 4 (x): PMC counters of the final MLA v3 decode (rows 64, ctx 4k) and GQA prefill v2 (ISL 5000)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for what in mla prefill; do
  if [ $what = mla ]; then ARGS="--mla-only --rows 64"; else ARGS="--ctx 5000"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d /tmp/pmc_${what}_a -- python3 $R/scripts/bench_attn.py $ARGS > $R/gpurun_out/r4x_${what}_a.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_${what}_b -- python3 $R/scripts/bench_attn.py $ARGS > $R/gpurun_out/r4x_${what}_b.log 2>&1 || exit $?
  mkdir -p $R/gpurun_out/pmc_r4x_$what && cp /tmp/pmc_${what}_a/*/*counter_collection.csv $R/gpurun_out/pmc_r4x_$what/a.csv && cp /tmp/pmc_${what}_b/*/*counter_collection.csv $R/gpurun_out/pmc_r4x_$what/b.csv
done
ls -la $R/gpurun_out/pmc_r4x_mla $R/gpurun_out/pmc_r4x_prefill
