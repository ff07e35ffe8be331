# round 4 (c): symm heap collectives incl. the fp8 EP dispatch and the chunked HT
# exchange, the hybrid KV manager with graphs, offload pack/unpack on the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_symm.py tests/test_hybrid_kv.py tests/test_offload.py tests/test_kvx_relay.py -q -x -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4c_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r4c_tests.log
[ $rc -ne 0 ] && grep -E "Error|error|FAILED|assert|mismatch|differ" gpurun_out/r4c_tests.log | head -30
exit $rc
