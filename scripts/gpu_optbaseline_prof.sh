# kernel profile of the optimized-baseline ladder's rate-8 stage (max-num-seqs 160) (one Qwen3-32B replica on one MI355X)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/ob_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ob_prof -o ob -- \
  python3 -u scripts/e2e_serving.py --model qwen3-32b --device cuda --replicas 1 --blocks 40000 \
  --configs prefix --system-len 6000 --question-len 1200 --output-len 360 --concurrency 160 \
  --workload guide_optimized-baseline_1.yaml \
  --overrides "load.stages=[{rate: 8, duration: 40}],data.shared_prefix.num_groups=19" \
  --out gpurun_out/ob_prof.json > gpurun_out/ob_prof.log 2>&1
rc=$?
grep "^\[e2e\]" gpurun_out/ob_prof.log | grep -v "\.\.\." | cut -c1-300
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/ob_prof/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f, f"total {tot/1e6:.1f} ms")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}% {r["Calls"]:>7} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
exit $rc
