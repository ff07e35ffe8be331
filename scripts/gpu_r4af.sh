# round 4 (af): the re-swept mgemm table (nt weight stream): numerics, 70B decode-only step, the driver's bench at its defaults
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mgemm.py tests/test_dgemm_table.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4af_t.log 2>&1 || { tail -20 gpurun_out/r4af_t.log; exit 1; }
tail -1 gpurun_out/r4af_t.log
timeout -k 10 300 python -u scripts/bench_decode.py --model llama-3-70b --batch 64 --isl 5000 --steps 60 > gpurun_out/r4af_d.log 2>&1 || { tail -20 gpurun_out/r4af_d.log; exit 1; }
grep 'decode batch' gpurun_out/r4af_d.log
timeout -k 10 600 python bench.py > gpurun_out/r4af_bench.out 2> gpurun_out/r4af_bench.err || { tail -20 gpurun_out/r4af_bench.err; exit 1; }
grep "timed step" gpurun_out/r4af_bench.err | tail -1; tail -1 gpurun_out/r4af_bench.out | cut -c1-300
