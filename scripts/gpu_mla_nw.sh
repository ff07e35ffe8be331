# MLA v2 at H=128: 8-wave (all heads, 256-register budget, spills) vs 4-wave (64-head workgroups, no spills).
set -o pipefail
mkdir -p gpurun_out
for nw in 8 4 8 4; do
  for kv in bf16 fp8; do
    LLMD_MLA_NW=$nw timeout -k 10 200 python -u scripts/bench_attn.py --mla --kv-dtype $kv > gpurun_out/mla_nw${nw}_$kv.log 2>&1 || { echo "mla bench failed"; tail -20 gpurun_out/mla_nw${nw}_$kv.log; exit 1; }
    echo "== NW=$nw kv=$kv"; grep "^mla" gpurun_out/mla_nw${nw}_$kv.log
  done
done
