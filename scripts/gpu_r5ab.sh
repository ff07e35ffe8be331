# Kernel times of the decode step with the fused reduce + add + RMSNorm (LLMD_MGEMM_NORM=1) vs the two-kernel path.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for arm in 1 0; do
  LLMD_MGEMM_NORM=$arm timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r5ab_$arm -o run -- python3 scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 30 > gpurun_out/r5ab_$arm.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r5ab_$arm.log; exit 1; }
  f=$(find /tmp/prof_r5ab_$arm -name '*kernel_trace.csv' | head -1)
  { echo "== norm=$arm"; grep "decode batch" gpurun_out/r5ab_$arm.log; python3 scripts/busy_from_trace.py "$f" 1.0 --breakdown; } | tee gpurun_out/r5ab_summary_$arm.txt
done
