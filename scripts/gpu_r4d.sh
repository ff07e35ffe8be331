# round 4 (d): the 1-GPU headline bench (driver's args) after the prefill-GEMM dispatch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r4d.out 2> gpurun_out/bench_r4d.err
rc=$?
tail -3 gpurun_out/bench_r4d.err
tail -1 gpurun_out/bench_r4d.out
exit $rc
