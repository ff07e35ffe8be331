set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_TRANS_F32 --output-format csv -d gpurun_out/pmc_attn -o p1 -- python3 scripts/attn_prefill_only.py > gpurun_out/pmc1.log 2>&1 || { echo pmc1 failed; tail -5 gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn -o p2 -- python3 scripts/attn_prefill_only.py > gpurun_out/pmc2.log 2>&1 || { echo pmc2 failed; tail -5 gpurun_out/pmc2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_attn/*counter_collection.csv")):
    agg = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "prefill_kernel" not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    print(f, {k: f"{v / max(1, n[k]):.4g}" for k, v in agg.items()})
PY
