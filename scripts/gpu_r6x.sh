# attention defaults (D128 V437, D64 V5): every prefill GPU test + gpt-oss model tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "prefill or gpt_oss or gptoss or attn" > gpurun_out/r6x_test.log 2>&1; rc=$?
tail -3 gpurun_out/r6x_test.log; exit $rc
