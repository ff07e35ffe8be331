# prefill attention v2 schedule variants A/B (5 default; 21 unpacked row sums; 37 buffer-descriptor DMA; 53 both; 117 53 + scalar mask branch)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/attn_v2_variants_ab.py --variants 5,21,37,53,117 --rounds 3 > gpurun_out/r6r.log 2>&1; rc=$?
grep -E "^AB|check|Error|error" gpurun_out/r6r.log; exit $rc
