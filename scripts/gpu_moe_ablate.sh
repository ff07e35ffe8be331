# fp8 MoE v3 ablation: full kernel vs no MFMA (DMA stream + barriers only) vs no refill DMA (MFMA on stale LDS)
set -o pipefail
mkdir -p gpurun_out/moeabl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 0 1 2; do
  LLMD_MOE_ABLATE=$a timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/moeabl/a$a -o run -- python3 scripts/moe_only.py gptoss > gpurun_out/moeabl/a$a.log 2>&1 || { echo "a$a failed"; tail -5 gpurun_out/moeabl/a$a.log; exit 1; }
  f=$(find gpurun_out/moeabl/a$a -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'moe_gemm3' in r['Name']: print('ablate $a', r['Name'][35:80], 'avg', round(float(r['AverageNs'])/1e3,1), 'us')
"
  find gpurun_out/moeabl/a$a -name "*kernel_trace.csv" -delete
done
