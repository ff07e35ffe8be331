# PMC counters of the block-fp8 grouped GEMM (moe_gemm3_fp8_kernel) at gpt-oss-120b and DeepSeek EP8 prefill shapes.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_moe
for s in gptoss deepseek; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_moe -o ${s}_p1 -- python3 scripts/moe_only.py $s > gpurun_out/pmc_moe1_$s.log 2>&1 || { echo pmc1 failed; tail -5 gpurun_out/pmc_moe1_$s.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_moe -o ${s}_p2 -- python3 scripts/moe_only.py $s > gpurun_out/pmc_moe2_$s.log 2>&1 || { echo pmc2 failed; tail -5 gpurun_out/pmc_moe2_$s.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pmc_moe -o ${s}_p3 -- python3 scripts/moe_only.py $s > gpurun_out/pmc_moe3_$s.log 2>&1 || { echo pmc3 failed; tail -5 gpurun_out/pmc_moe3_$s.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_moe -o ${s}_kt -- python3 scripts/moe_only.py $s > gpurun_out/pmc_moe4_$s.log 2>&1 || { echo kt failed; tail -5 gpurun_out/pmc_moe4_$s.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_moe/*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        kn = r.get("Kernel_Name", "")
        if "moe_gemm3_fp8" not in kn:
            continue
        tag = "gemm1(act)" if "ILi1E" in kn else "gemm2"
        agg[tag][r["Counter_Name"]] += float(r["Counter_Value"])
        n[tag][r["Counter_Name"]] += 1
    for tag in sorted(agg):
        print(f.split("/")[-1], tag, {k: f"{v / max(1, n[tag][k]):.4g}" for k, v in sorted(agg[tag].items())})
for f in sorted(glob.glob("gpurun_out/pmc_moe/*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "moe" in r["Name"] or "quant" in r["Name"]:
            print("stats", f.split("/")[-1][:12], r["Name"][:48], r["Calls"], r["AverageNs"])
PY
grep -h "TF/s" gpurun_out/pmc_moe4_*.log
