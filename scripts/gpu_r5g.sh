# the driver's bench with the round-5 prefill GEMMs (pgemm table + whole-prompt 5064-token steps), then the
# kernel breakdown of the same run under rocprofv3
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5g_bench.out 2> gpurun_out/r5g_bench.err
rc=$?
tail -3 gpurun_out/r5g_bench.err; cat gpurun_out/r5g_bench.out
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/r5g_prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g_prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5g_prof.out 2> gpurun_out/r5g_prof.err
rc=$?
tail -2 gpurun_out/r5g_prof.err
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob("gpurun_out/r5g_prof/*kernel_stats.csv"):
    rows += list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# total kernel time {tot / 1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e6:10.1f} ms {100 * t / tot:5.1f}% {int(r['Calls']):7d} calls avg {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:110]}")
PY
exit $rc
