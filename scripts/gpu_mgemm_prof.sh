# Kernel-trace stats of the medium-M decode GEMM's best plans (GEMM vs split-K reduce time).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_mgemm
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_mgemm -o run -- python3 scripts/mgemm_prof.py > gpurun_out/mgemm_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/mgemm_prof.log; exit 1; }
f=$(find gpurun_out/prof_mgemm -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r.get("Grid_Size", r.get("Grid_Size_X", ""))) for r in rows
       if "mgemm" in r["Kernel_Name"]]
# group consecutive runs of 40 calls per shape: kernel + reduce alternate
agg = collections.OrderedDict()
shape = -1; prev = None
for name, dur, grid in seq:
    k = ("reduce" if "reduce" in name else "gemm")
    key = name.split("(")[0][-60:]
    agg.setdefault(key, []).append(dur)
for k, v in agg.items():
    v = sorted(v)[len(v)//10: -max(1, len(v)//10)]
    print(f"{k:60s} n={len(v):4d} median {sorted(v)[len(v)//2]/1000:7.1f} us mean {sum(v)/len(v)/1000:7.1f} us")
PY
