# per-kernel breakdown of moe_experts_fp8 at the gpt-oss / DeepSeek prefill shapes
set -o pipefail
mkdir -p gpurun_out/moeprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for sh in gptoss deepseek; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/moeprof/$sh -o run -- python3 scripts/moe_only.py $sh > gpurun_out/moeprof/$sh.log 2>&1 || { echo "prof $sh failed"; tail -5 gpurun_out/moeprof/$sh.log; exit 1; }
  grep -h "T=" gpurun_out/moeprof/$sh.log
  f=$(find gpurun_out/moeprof/$sh -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:8]:
    print('  %-60s n=%5s avg=%8.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
done
find gpurun_out/moeprof -name "*kernel_trace.csv" -delete; find gpurun_out/moeprof -name "*.db" -delete
