# round 4 (ag): DeepSeek-R1 one-EP-rank decode projection again with the nt decode-stream defaults (mgemm, MoE v2 experts)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/bench_wide_ep_rank.py --steps 20 --out gpurun_out/r4ag_wide_ep_rank.json > gpurun_out/r4ag_wide_ep_rank.log 2>&1 || { tail -20 gpurun_out/r4ag_wide_ep_rank.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4ag_wide_ep_rank.log | tail -4
