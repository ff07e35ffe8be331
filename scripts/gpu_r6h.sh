# Round 6: medium-M decode GEMM at 129-256 rows - numerics, then plan sweeps at M 192 / 256 (bf16 and fp8).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_mgemm.py tests/test_kernels_gpu.py -k "mgemm" > gpurun_out/r6h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6h_tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "llama-3-70b 1 qkv o gate_up down" "llama-3-70b 2 qkv o gate_up down" "llama-3-8b 1 qkv o gate_up down" "gpt-oss-120b 1 qkv o"; do
  set -- $spec; m=$1; tp=$2; shift 2
  timeout -k 10 600 python -u scripts/sweep_mgemm.py --model $m --tp $tp --m 192 256 --iters 20 --names "$@" > gpurun_out/r6h_sweep_${m}_tp${tp}.log 2>&1
  rc=$?; grep -E "hipBLASLt" gpurun_out/r6h_sweep_${m}_tp${tp}.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
