# gpt-oss-120b serving after K-step-major MXFP4 scales: 60-step windows, mxfp4 then fp8, same box
set -o pipefail
mkdir -p gpurun_out
for q in mxfp4 fp8; do
timeout -k 10 540 python3 bench.py --model gpt-oss-120b --isl 5150 --osl 250 --quantization $q --concurrency 256 --steps 60 --warmup 10 --fp8-extra off > gpurun_out/r6ay_$q.log 2>&1 || { tail -20 gpurun_out/r6ay_$q.log; exit 1; }
grep '"metric"' gpurun_out/r6ay_$q.log | cut -c1-200
done
