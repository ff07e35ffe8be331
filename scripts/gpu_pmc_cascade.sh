# PMC counters of the shared-prefix decode kernels (one pass per counter group), then a
# kernel-trace busy breakdown of the 70B bench with the current code
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_sp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_sp -o p1 -- python3 scripts/shared_prefix_only.py > gpurun_out/pmc_sp1.log 2>&1 || { echo p1 failed; tail -5 gpurun_out/pmc_sp1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sp -o p2 -- python3 scripts/shared_prefix_only.py > gpurun_out/pmc_sp2.log 2>&1 || { echo p2 failed; tail -5 gpurun_out/pmc_sp2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_sp -o p3 -- python3 scripts/shared_prefix_only.py > gpurun_out/pmc_sp3.log 2>&1 || { echo p3 failed; tail -5 gpurun_out/pmc_sp3.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_sp -o p4 -- python3 scripts/shared_prefix_only.py > gpurun_out/pmc_sp4.log 2>&1 || { echo p4 failed; tail -5 gpurun_out/pmc_sp4.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_sp -o kt -- python3 scripts/shared_prefix_only.py > gpurun_out/pmc_sp5.log 2>&1 || { echo kt failed; tail -5 gpurun_out/pmc_sp5.log; exit 1; }
grep "bytes" gpurun_out/pmc_sp5.log
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_sp/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        key = "prefix_v2" if "shared_prefix_v2" in k else "suffix" if "paged_decode_kernel" in k else "reduce" if "decode_reduce" in k else None
        if key is None:
            continue
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"]); n[key][r["Counter_Name"]] += 1
    for key in agg:
        print(f.split("/")[-1][:24], key, {c: f"{v / max(1, n[key][c]):.4g}" for c, v in sorted(agg[key].items())})
for f in sorted(glob.glob("gpurun_out/pmc_sp/**/*kernel_stats.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        print("stats", r["Name"][:70], r["Calls"], r["AverageNs"])
PY
bash scripts/gpu_busy.sh
