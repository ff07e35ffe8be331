# Prefill step shape A/B on the driver's bench: whole-prompt 5063-token steps (default: align 512, final
# chunk kept whole) vs 4096-token steps + a 1030-token tail step (align 2048, final chunks trimmed too).
set -o pipefail
mkdir -p gpurun_out
for arm in base a2048 base a2048; do
  if [ $arm = base ]; then envs=""; else envs="LLMD_PREFILL_ALIGN=2048 LLMD_ALIGN_KEEP_FINAL=0"; fi
  env $envs timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5z_$arm.log 2>&1
  rc=$?; echo "== $arm"; grep -E "timed step sizes" gpurun_out/r5z_$arm.log; grep -o '"value": [0-9.]*' gpurun_out/r5z_$arm.log
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r5z_$arm.log; exit $rc; }
done
exit 0
