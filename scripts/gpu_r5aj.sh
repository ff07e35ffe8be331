# Llama-3-8B with its medium-M decode GEMM rows in ops/mgemm_table.py (so the decode fusions apply too):
# mgemm numerics, decode step, aggregated bench at 64 / 256 in flight.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_mgemm.py > gpurun_out/r5aj_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5aj_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-8b --batch 64 --isl 5000 --steps 40 > gpurun_out/r5aj_8b_dec.log 2>&1
rc=$?; grep "decode batch" gpurun_out/r5aj_8b_dec.log; [ $rc -ne 0 ] && exit $rc
for c in 64 256; do
  timeout -k 10 400 python -u bench.py --model llama-3-8b --concurrency $c --steps 40 --warmup 10 > gpurun_out/r5aj_8b_c$c.log 2>&1
  rc=$?; echo "== c$c"; grep -E "timed step sizes" gpurun_out/r5aj_8b_c$c.log; grep -o '"value": [0-9.]*\|"p50_ttft_s": [0-9.]*' gpurun_out/r5aj_8b_c$c.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/r5aj_8b_c$c.log; exit $rc; }
done
exit 0
