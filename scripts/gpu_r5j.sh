# Decode fusions: mgemm split-K fixup in the kernel and the SiLU-and-mul in the
# gate/up GEMM's epilogue - numerics, then the 70B decode step A/B (batch 64, ctx 5000) and its
# kernel breakdown, then the driver bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_mgemm.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "mgemm" > gpurun_out/r5j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5j_tests.log; [ $rc -ne 0 ] && exit $rc
# prefill attention v4 (32x32x16): numerics, then the A/B against v2
timeout -k 10 300 python -u -m pytest tests/test_prefill_v4.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5j_attn_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r5j_attn_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/attn_v4_ab.py > gpurun_out/r5j_attn_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5j_attn_ab.log | grep "AB\|check"; [ $rc -ne 0 ] && exit $rc
for cfg in "0 0" "1 0" "1 1"; do
  set -- $cfg
  LLMD_MGEMM_FIXUP=$1 LLMD_MGEMM_SILU=$2 timeout -k 10 400 python -u scripts/bench_decode.py --steps 40 > gpurun_out/r5j_dec_$1$2.log 2>&1
  rc=$?; echo "fixup=$1 silu=$2: $(grep -v amdgpu.ids gpurun_out/r5j_dec_$1$2.log | tail -1)"; [ $rc -ne 0 ] && exit $rc
done
rm -rf gpurun_out/r5j_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5j_prof -o dec -- python3 scripts/bench_decode.py --steps 40 > gpurun_out/r5j_prof.out 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r5j_prof.out; exit $rc; }
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob("gpurun_out/r5j_prof/*kernel_stats.csv"):
    rows += list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# total kernel time {tot / 1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e6:10.1f} ms {100 * t / tot:5.1f}% {int(r['Calls']):7d} calls avg {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:100]}")
PY
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5j_bench.out 2> gpurun_out/r5j_bench.err
rc=$?; grep "timed step" gpurun_out/r5j_bench.err; cat gpurun_out/r5j_bench.out; exit $rc
