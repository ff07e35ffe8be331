# --quantization mxfp4 (MXFP4 experts) in the engine: GPU test, then gpt-oss-120b serving mxfp4 (kernel split) vs fp8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine.py -k mxfp4 > gpurun_out/r6ad_test.log 2>&1 || { tail -40 gpurun_out/r6ad_test.log; exit 1; }
tail -2 gpurun_out/r6ad_test.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/r6ad_prof -o run -- python3 bench.py --model gpt-oss-120b --isl 5150 --osl 250 --quantization mxfp4 --concurrency 256 --steps 20 --warmup 5 --fp8-extra off > gpurun_out/r6ad.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r6ad.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 gpurun_out/r6ad.log; exit $rc; }
f=$(find gpurun_out/r6ad_prof -name "*results.db" -o -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_window.py "$f" 1.6 30 > gpurun_out/r6ad_window.txt && cat gpurun_out/r6ad_window.txt
rm -f "$f"
timeout -k 10 420 python3 bench.py --model gpt-oss-120b --isl 5150 --osl 250 --quantization fp8 --concurrency 256 --steps 20 --warmup 5 --fp8-extra off > gpurun_out/r6ad_fp8.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r6ad_fp8.log | cut -c1-300; exit $rc
