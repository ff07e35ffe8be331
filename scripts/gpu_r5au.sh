# Paged decode at head dim 64 (gpt-oss) vs 128 (70B), and a split-count sweep at D = 64.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probe_decode_d64.py > gpurun_out/r5au_d64.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5au_d64.log; exit $rc
