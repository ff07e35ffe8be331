# round 4 (e): headline bench A/B on one box: prefill-GEMM autotune off, then on
set -o pipefail
mkdir -p gpurun_out
LLMD_PGEMM_AUTO=0 timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_auto0.out 2> gpurun_out/bench_auto0.err
rc=$?
grep "timed step" gpurun_out/bench_auto0.err; tail -1 gpurun_out/bench_auto0.out | cut -c1-200
[ $rc -ne 0 ] && exit $rc
LLMD_PGEMM_VERBOSE=1 timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_auto1.out 2> gpurun_out/bench_auto1.err
rc=$?
grep "timed step" gpurun_out/bench_auto1.err; tail -1 gpurun_out/bench_auto1.out | cut -c1-200
grep -i "prefill GEMM" gpurun_out/bench_auto1.err | head -20
[ $rc -ne 0 ] && exit $rc
[ $rc -ne 0 ] && exit $rc
LLMD_ALIGN_KEEP_FINAL=1 timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_keepfinal.out 2> gpurun_out/bench_keepfinal.err
rc=$?
grep "timed step" gpurun_out/bench_keepfinal.err; tail -1 gpurun_out/bench_keepfinal.out | cut -c1-200
[ $rc -ne 0 ] && exit $rc
exit $rc
