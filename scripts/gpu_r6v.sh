# software-pipelined prefill attention v5: numerics, then A/B against v2 (V5 / V53)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_prefill_v5.py > gpurun_out/r6v_test.log 2>&1 || { tail -40 gpurun_out/r6v_test.log; exit 1; }
tail -2 gpurun_out/r6v_test.log
timeout -k 10 600 python -u scripts/attn_v2_variants_ab.py --variants 5,53,v5 --rounds 3 > gpurun_out/r6v_ab.log 2>&1; rc=$?
grep -E "^AB|check|Error|error" gpurun_out/r6v_ab.log; exit $rc
