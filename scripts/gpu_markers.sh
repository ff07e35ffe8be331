# roctx engine-phase ranges in a rocprofv3 marker + kernel trace (8B decode, small batch).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_mk
LLMD_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/prof_mk -o run -- python3 scripts/bench_decode.py --model llama-3-8b --batch 16 --isl 1000 --steps 20 > gpurun_out/markers.log 2>&1 || { echo "marker prof failed"; tail -20 gpurun_out/markers.log; exit 1; }
ls gpurun_out/prof_mk
f=$(find gpurun_out/prof_mk -name '*marker_api_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
print("columns:", list(rows[0].keys()) if rows else None)
d = collections.defaultdict(list)
for r in rows:
    name = r.get("Message") or r.get("Marker_Name") or r.get("Function") or ""
    try:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    except (KeyError, ValueError):
        continue
    d[name.split(" ")[0]].append(dur)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k:24s} n={len(v):5d} median {v[len(v)//2]:9.1f} us  total {sum(v)/1000:9.1f} ms")
PY
find gpurun_out/prof_mk -name '*kernel_trace.csv' -delete
