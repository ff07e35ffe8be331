# MFMA rate by operand format (probe), then PMC counters of the MXFP4 / fp8 MoE tile GEMMs at T=5405
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/probes/mfma_rate_probe > gpurun_out/r6af_rate.txt 2>&1 || { cat gpurun_out/r6af_rate.txt; exit 1; }
cat gpurun_out/r6af_rate.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_r6af
for kind in mxfp4 fp8; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_r6af -o ${kind}_p1 -- python3 scripts/mxfp4_only.py $kind > gpurun_out/r6af_1_$kind.log 2>&1 || { echo pmc1 failed; tail -5 gpurun_out/r6af_1_$kind.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_r6af -o ${kind}_p2 -- python3 scripts/mxfp4_only.py $kind > gpurun_out/r6af_2_$kind.log 2>&1 || { echo pmc2 failed; tail -5 gpurun_out/r6af_2_$kind.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_r6af -o ${kind}_p3 -- python3 scripts/mxfp4_only.py $kind > gpurun_out/r6af_3_$kind.log 2>&1 || { echo pmc3 failed; tail -5 gpurun_out/r6af_3_$kind.log; exit 1; }
done
python3 - <<'PY' > gpurun_out/r6af_pmc.txt
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_r6af/*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        kn = r.get("Kernel_Name", "")
        if "moe_gemm8" not in kn:
            continue
        tag = kn.split("(")[0].split("::")[-1]
        agg[tag][r["Counter_Name"]] += float(r["Counter_Value"])
        n[tag][r["Counter_Name"]] += 1
    for tag in sorted(agg):
        print(f.split("/")[-1].split("_counter")[0], tag, {k: f"{v / max(1, n[tag][k]):.4g}" for k, v in sorted(agg[tag].items())})
PY
cat gpurun_out/r6af_pmc.txt
