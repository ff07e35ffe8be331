# moe8 work-item order A/B (0: XCD chunks, 1: round-robin)
set -o pipefail
mkdir -p gpurun_out
for o in 0 1; do
  LLMD_MOE8_ORDER=$o VERS=8 timeout -k 10 200 python -u scripts/moe_tile_overhead.py > gpurun_out/r6l_ovh_$o.log 2>&1 || { cat gpurun_out/r6l_ovh_$o.log; exit 1; }
  echo "order $o"; cat gpurun_out/r6l_ovh_$o.log
  LLMD_MOE8_ORDER=$o timeout -k 10 300 python -u scripts/bench_moe8.py > gpurun_out/r6l_bench_$o.log 2>&1 || { cat gpurun_out/r6l_bench_$o.log; exit 1; }
  cat gpurun_out/r6l_bench_$o.log
done
