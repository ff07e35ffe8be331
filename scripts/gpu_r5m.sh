# mgemm split-K fixup, same-XCD form (no fences): numerics with the switch on, then the decode A/B.
set -o pipefail
mkdir -p gpurun_out
LLMD_MGEMM_FIXUP=1 timeout -k 10 300 python -u -m pytest tests/test_mgemm.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5m_tests_fix.log 2>&1
rc=$?; tail -2 gpurun_out/r5m_tests_fix.log; [ $rc -ne 0 ] && exit $rc
for f in 0 1 0 1; do
  LLMD_MGEMM_FIXUP=$f timeout -k 10 400 python -u scripts/bench_decode.py --steps 40 > gpurun_out/r5m_dec_$f.log 2>&1
  rc=$?; echo "fixup=$f: $(grep -v amdgpu.ids gpurun_out/r5m_dec_$f.log | tail -1)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
