"""TunableOp search for the fp8 W8A8 projections (torch._scaled_mm with row-wise
scales: per-token activation scales, per-channel weight scales - ops.fp8_linear)
at a preset's serving shapes, then default vs tuned. Results merge into the
committed table (scripts/merge_tunableop.py) that the engine loads in lookup-only
mode. Weights rotate through > 1 GB so the 256 MB Infinity Cache does not
flatter decode GEMMs.
  python scripts/tune_fp8_gemm.py --models llama-3-70b --ms 64 128 --out gpurun_out/tunableop_fp8.csv"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd.ops.gemm_tuning import model_gemm_shapes  # noqa: E402

F8 = torch.float8_e4m3fn


def operands(M, N, K, nb):
    ws = [(torch.randn(N, K, device="cuda") * 0.05).to(F8) for _ in range(nb)]
    wsc = torch.rand(1, N, device="cuda") * 0.01 + 0.001
    x = (torch.randn(M, K, device="cuda")).to(F8)
    xs = torch.rand(M, 1, device="cuda") * 0.01 + 0.001
    return ws, wsc, x, xs


def timed(M, N, K, iters=30):
    nb = max(2, (1 << 30) // (N * K) + 1)
    ws, wsc, x, xs = operands(M, N, K, nb)
    f = lambda i: torch._scaled_mm(x, ws[i % nb].t(), scale_a=xs, scale_b=wsc, out_dtype=torch.bfloat16)  # noqa
    for i in range(3):
        f(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        f(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="*", default=["llama-3-70b"])
    ap.add_argument("--ms", type=int, nargs="*", default=[1, 8, 16, 32, 64, 128, 256, 512, 4608])
    ap.add_argument("--duration-ms", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/tunableop_fp8.csv")
    ap.add_argument("--names", nargs="*", default=["qkv", "o", "gate_up", "down"])
    a = ap.parse_args()
    shapes = [(m, n, M, N, K) for m in a.models for n, (N, K) in model_gemm_shapes(m).items() if n in a.names
              for M in a.ms]
    base = {s: timed(*s[2:]) for s in shapes}
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_rotating_buffer_size(512)
    tun.set_max_tuning_duration(a.duration_ms)
    tun.set_filename(a.out)
    t0 = time.time()
    for s in shapes:
        M, N, K = s[2:]
        ws, wsc, x, xs = operands(M, N, K, 1)
        torch._scaled_mm(x, ws[0].t(), scale_a=xs, scale_b=wsc, out_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        print(f"tuned {s} at {time.time() - t0:.0f}s", flush=True)
    tot0 = tot1 = 0.0
    for s in shapes:
        m, name, M, N, K = s
        t1 = timed(M, N, K)
        tot0 += base[s]
        tot1 += t1
        by = N * K
        print(f"{m:12s} {name:8s} M={M:5d}: default {base[s] * 1e6:8.1f} us {by / base[s] / 1e12:5.2f} TB/s | "
              f"tuned {t1 * 1e6:8.1f} us {by / t1 / 1e12:5.2f} TB/s", flush=True)
    print(f"total default {tot0 * 1e3:.3f} ms tuned {tot1 * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
