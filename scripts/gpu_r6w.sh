# v2 attention variants 181 / 309 / 437 (pre-scaled Q + accumulator start at -m; MFMA row sums): numerics, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_prefill_v5.py -k "variants" > gpurun_out/r6w_test.log 2>&1 || { tail -40 gpurun_out/r6w_test.log; exit 1; }
tail -2 gpurun_out/r6w_test.log
timeout -k 10 600 python -u scripts/attn_v2_variants_ab.py --variants 53,181,309,437 --rounds 3 > gpurun_out/r6w_ab.log 2>&1; rc=$?
grep -E "^AB|check|Error|error" gpurun_out/r6w_ab.log; exit $rc
