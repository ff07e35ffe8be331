# PMC counters of the MoE v4 grouped GEMMs (csrc/ops/moe4.hip, bf16 and block-fp8) at DeepSeek EP8 and
# gpt-oss-120b prefill shapes: one counter pass per rocprofv3 run (hardware limits per block respected).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_moe4
for s in deepseek gptoss; do
for dt in fp8 bf16; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_moe4 -o ${s}_${dt}_p1 -- python3 scripts/moe_only.py $s $dt > gpurun_out/pmc_moe4_1_$s$dt.log 2>&1 || { echo pmc1 failed; tail -5 gpurun_out/pmc_moe4_1_$s$dt.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_moe4 -o ${s}_${dt}_p2 -- python3 scripts/moe_only.py $s $dt > gpurun_out/pmc_moe4_2_$s$dt.log 2>&1 || { echo pmc2 failed; tail -5 gpurun_out/pmc_moe4_2_$s$dt.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_moe4 -o ${s}_${dt}_kt -- python3 scripts/moe_only.py $s $dt > gpurun_out/pmc_moe4_3_$s$dt.log 2>&1 || { echo kt failed; tail -5 gpurun_out/pmc_moe4_3_$s$dt.log; exit 1; }
done
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_moe4/*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        kn = r.get("Kernel_Name", "")
        if "moe_gemm4" not in kn:
            continue
        tag = ("fp8 " if "fp8" in kn else "bf16 ") + ("gemm1(act)" if ("<1," in kn or "ILi1E" in kn) else "gemm2")
        agg[tag][r["Counter_Name"]] += float(r["Counter_Value"])
        n[tag][r["Counter_Name"]] += 1
    for tag in sorted(agg):
        print(f.split("/")[-1], tag, {k: f"{v / max(1, n[tag][k]):.4g}" for k, v in sorted(agg[tag].items())})
for f in sorted(glob.glob("gpurun_out/pmc_moe4/*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "moe" in r["Name"] or "quant" in r["Name"]:
            print("stats", f.split("/")[-1][:16], r["Name"][:56], r["Calls"], r["AverageNs"])
PY
grep -h "TF/s" gpurun_out/pmc_moe4_3_*.log
