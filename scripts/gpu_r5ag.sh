# Host-side profile of 20 decode steps (70B, batch 64): where the ~1.1 ms of per-step GPU idle goes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 20 --host-profile > gpurun_out/r5ag_host.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5ag_host.log | tail -45; exit $rc
