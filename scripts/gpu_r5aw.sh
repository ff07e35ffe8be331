# Host time between decode graph replays on the bench (scripts/host_gap_gpu.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/host_gap_gpu.py --steps 20 --warmup 5 > gpurun_out/r5aw_gap.log 2>&1
rc=$?; grep -E "^\[gap\]|timed step|^\{" gpurun_out/r5aw_gap.log | cut -c1-200; exit $rc
