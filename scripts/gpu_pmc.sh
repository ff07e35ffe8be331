# PMC counters of the prefill attention kernel (ISL 5000, 70B heads); one pass per counter group.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_attn
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_TRANS_F32 --output-format csv -d gpurun_out/pmc_attn -o p1 -- python3 scripts/attn_prefill_only.py > gpurun_out/pmc1.log 2>&1 || { echo pmc1 failed; tail -5 gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn -o p2 -- python3 scripts/attn_prefill_only.py > gpurun_out/pmc2.log 2>&1 || { echo pmc2 failed; tail -5 gpurun_out/pmc2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_attn -o kt -- python3 scripts/attn_prefill_only.py > gpurun_out/pmc3.log 2>&1 || { echo kt failed; tail -5 gpurun_out/pmc3.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_attn/*counter_collection.csv")):
    agg = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "prefill" not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    print(f.split("/")[-1], {k: f"{v / max(1, n[k]):.4g}" for k, v in sorted(agg.items())})
for f in sorted(glob.glob("gpurun_out/pmc_attn/*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "prefill" in r["Name"]:
            print("stats", r["Name"][:60], r["Calls"], r["AverageNs"])
PY
grep -h "TF/s" gpurun_out/pmc3.log | tail -1
