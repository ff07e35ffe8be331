# The P/D prefill rank's job with the round-5 kernels: prefill-only throughput at ISL 5000 (8192-token steps).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/bench_prefill_rate.py --steps 16 > gpurun_out/r5af_prefill_rate.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5af_prefill_rate.log | tail -4; exit $rc
