# gpt-oss decode attention (D 64, 64 q / 8 kv heads): time vs KV split count at serving batch sizes
set -o pipefail
mkdir -p gpurun_out
NSPLIT_D=64 NSPLIT_CASES=256:5200,128:5200,64:5200,256:2600 timeout -k 10 300 python -u scripts/bench_decode_nsplit.py > gpurun_out/r6aq.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6aq.log | tail -6
NSPLIT_CASES=64:5125 timeout -k 10 200 python -u scripts/bench_decode_nsplit.py >> gpurun_out/r6aq.log 2>&1 || exit 1
tail -1 gpurun_out/r6aq.log; exit $rc
