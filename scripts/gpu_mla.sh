# MLA: DeepSeek/MLA GPU tests, then the MLA microbenchmark (bf16 and fp8 latent cache).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_deepseek.py tests/test_fp8_kv.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/mla_tests.log 2>&1 || { echo "mla tests failed"; tail -40 gpurun_out/mla_tests.log; exit 1; }
tail -1 gpurun_out/mla_tests.log
for kv in bf16 fp8; do
  timeout -k 10 200 python -u scripts/bench_attn.py --mla --kv-dtype $kv > gpurun_out/mla_$kv.log 2>&1 || { echo "mla bench failed"; tail -20 gpurun_out/mla_$kv.log; exit 1; }
  grep "^mla" gpurun_out/mla_$kv.log
done
