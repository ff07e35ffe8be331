# Round-5 final-code rehearsal of the driver's multi-GPU bench topologies on ONE GPU (scripts/gpu_scale_rehearsal.sh),
# then the MoE v4 PMC passes (scripts/gpu_pmc_moe4.sh).
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_scale_rehearsal.sh || exit 1
bash scripts/gpu_pmc_moe4.sh
