# D = 64 (gpt-oss) v2 attention variants: numerics, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_prefill_v5.py -k "d64" > gpurun_out/r6y_test.log 2>&1 || { tail -40 gpurun_out/r6y_test.log; exit 1; }
tail -2 gpurun_out/r6y_test.log
AB_D64=1 timeout -k 10 600 python -u scripts/attn_v2_variants_ab.py --variants 5,53,181,437 --rounds 3 > gpurun_out/r6y_ab.log 2>&1; rc=$?
grep -E "^AB|check|Error|error" gpurun_out/r6y_ab.log; exit $rc
