# PMC counters of hipBLASLt vs the pgemm variants on one prefill GEMM shape; one pass per counter group
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_pgemm
rm -rf $OUT
ARGS="${PGEMM_PMC_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES --output-format csv -d $OUT -o p1 -- python3 scripts/pgemm_pmc_one.py $ARGS > gpurun_out/pgpmc1.log 2>&1 || { echo pmc1 failed; tail -5 gpurun_out/pgpmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $OUT -o p2 -- python3 scripts/pgemm_pmc_one.py $ARGS > gpurun_out/pgpmc2.log 2>&1 || { echo pmc2 failed; tail -5 gpurun_out/pgpmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY --output-format csv -d $OUT -o p3 -- python3 scripts/pgemm_pmc_one.py $ARGS > gpurun_out/pgpmc3.log 2>&1 || { echo pmc3 failed; tail -5 gpurun_out/pgpmc3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- python3 scripts/pgemm_pmc_one.py $ARGS > gpurun_out/pgpmc4.log 2>&1 || { echo kt failed; tail -5 gpurun_out/pgpmc4.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
def kind(n):
    if "Cijk" in n:
        return "blas"
    for v in ("pgemm6", "pgemm5", "pgemm4"):
        if v in n:
            return v
    return "pgemm0" if "pgemm_kernel" in n else None
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in sorted(glob.glob("gpurun_out/pmc_pgemm/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = kind(r.get("Kernel_Name", ""))
        if k is None:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k in sorted(agg):
    print(k, {c: f"{v / max(1, cnt[k][c]):.5g}" for c, v in sorted(agg[k].items())})
for f in sorted(glob.glob("gpurun_out/pmc_pgemm/*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        k = kind(r["Name"])
        if k:
            print("stats", k, r["Name"][:90], r["Calls"], r["AverageNs"])
PY
