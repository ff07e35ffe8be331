"""Prefill GEMM efficiency at the token counts a continuous-batching step
really produces (decode rows + a partial prefill chunk, so M is rarely a
multiple of the tile): hipBLASLt at M as-is vs M padded up to a multiple of
256, useful TF/s (2*M*N*K / t) for both.  Llama-3-70B TP1 shapes.
  python scripts/bench_gemm_oddm.py [--lookup] [--m ...]"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)}


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="*", default=[1100, 2112, 3064, 4100, 5064, 6000, 7000, 8192, 8256])
    ap.add_argument("--lookup", action="store_true")
    a = ap.parse_args()
    if a.lookup:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from llmd_amd.ops.gemm_tuning import enable_lookup
        print("lookup:", enable_lookup())
    dev = "cuda"
    ws = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in SHAPES.items()}
    tot = {}
    for M in a.m:
        Mp = (M + 255) // 256 * 256
        x = torch.randn(Mp, 8192, device=dev, dtype=torch.bfloat16)
        xf = torch.randn(Mp, 28672, device=dev, dtype=torch.bfloat16)
        ta = tp = 0.0
        for name, (N, K) in SHAPES.items():
            src = xf if K == 28672 else x
            t1 = timeit(lambda: F.linear(src[:M], ws[name]))
            t2 = timeit(lambda: F.linear(src[:Mp], ws[name]))
            fl = 2.0 * M * N * K
            ta += t1
            tp += t2
            print(f"M={M:5d} (pad {Mp:5d}) {name:8s}: as-is {t1 * 1e3:7.3f} ms {fl / t1 / 1e12:7.1f} TF/s | "
                  f"padded {t2 * 1e3:7.3f} ms {fl / t2 / 1e12:7.1f} TF/s", flush=True)
        tot[M] = (ta, tp)
        print(f"M={M:5d} layer total: as-is {ta * 1e3:.3f} ms, padded {tp * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
