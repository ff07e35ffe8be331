set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "sample" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sample_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sample_test.log; exit 1; }
tail -1 gpurun_out/sample_test.log
timeout -k 10 120 python - <<'PY'
import time, torch, sys, os
sys.path.insert(0, os.getcwd())
from llmd_amd import ops
for B, V in ((1, 151936), (8, 151936), (32, 151936), (110, 151936), (256, 151936), (64, 201088), (64, 128256)):
    lg = torch.randn(B, V, device="cuda").to(torch.bfloat16)
    t = torch.full((B,), 0.7, device="cuda"); s = torch.arange(B, device="cuda", dtype=torch.int64)
    for _ in range(3): ops.sample(lg, t, s)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(50): ops.sample(lg, t, s)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 50
    print(f"sample B={B:4d} V={V}: {dt * 1e6:7.1f} us ({B * V * 2 / dt / 1e9:6.0f} GB/s)")
PY
