# Energy per FLOP of the bf16 MFMA shapes at the power cap (scripts/mfma_energy.py, register-only streams).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/mfma_energy.py > gpurun_out/r5y_mfma_energy.log 2>&1
rc=$?; grep "TF/s" gpurun_out/r5y_mfma_energy.log; exit $rc
