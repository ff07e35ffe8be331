# PMC of the GQA prefill attention v2 variants V5 (round-5 default) and V53 (round-6 default) at ISL 5000
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_attn
for v in 5 53; do
LLMD_PREFILL_V2_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_attn -o v${v}_p1 -- python3 scripts/attn_only.py 10 > gpurun_out/pmc_attn_1_$v.log 2>&1 || { echo pmc1 failed; tail -5 gpurun_out/pmc_attn_1_$v.log; exit 1; }
LLMD_PREFILL_V2_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn -o v${v}_p2 -- python3 scripts/attn_only.py 10 > gpurun_out/pmc_attn_2_$v.log 2>&1 || { echo pmc2 failed; tail -5 gpurun_out/pmc_attn_2_$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_attn/*counter_collection.csv")):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "prefill_v2" not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[-1], {k: f"{v / max(1, n[k]):.4g}" for k, v in sorted(agg.items())})
PY
