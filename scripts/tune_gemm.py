"""Offline GEMM selection for the serving shapes with PyTorch TunableOp
(hipBLASLt + rocBLAS solution search), then an A/B of default vs tuned.

The engine loads the resulting CSV in lookup-only mode (llmd_amd/ops/gemm_tuning.py),
so no tuning ever happens inside a served step or a graph capture.
  python scripts/tune_gemm.py [--models llama-3-70b] [--ms 1 8 16 32 64 128] [--out FILE]

Weights rotate through > 512 MB of copies while timing so the 256 MB
Infinity Cache does not flatter small matrices (decode GEMMs are HBM streams).
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmd_amd.ops.gemm_tuning import model_gemm_shapes  # noqa: E402


def timed(M, N, K, iters=30):
    nb = max(2, (1 << 30) // (N * K * 2) + 1)
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(nb)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    for i in range(3):
        F.linear(x, ws[i % nb])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        F.linear(x, ws[i % nb])
    torch.cuda.synchronize()
    del ws
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="*", default=["llama-3-70b"])
    ap.add_argument("--ms", type=int, nargs="*", default=[1, 2, 4, 8, 16, 32, 64, 128])
    ap.add_argument("--duration-ms", type=int, default=10)
    ap.add_argument("--tp", type=int, default=1, help="shapes of one rank of a TP-N replica")
    ap.add_argument("--out", default="gpurun_out/tunableop_gfx950.csv")
    ap.add_argument("--names", nargs="*", default=None,
                    help="subset of qkv/o/gate_up/down/lm_head (prefill M: lm_head only sees sampled rows)")
    a = ap.parse_args()
    shapes = []
    for m in a.models:
        for name, (N, K) in model_gemm_shapes(m, tp=a.tp).items():
            if a.names and name not in a.names:
                continue
            for M in a.ms:
                shapes.append((m, name, M, N, K))
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
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        F.linear(x, w)
        torch.cuda.synchronize()
        print(f"tuned {s} at {time.time() - t0:.0f}s", flush=True)
    # TunableOp writes the file when the process exits; tuning stays enabled so
    # the A/B below re-uses the in-memory results without re-tuning.
    tot0 = tot1 = 0.0
    for s in shapes:
        m, name, M, N, K = s
        t1 = timed(M, N, K)
        tot0 += base[s]
        tot1 += t1
        by = N * K * 2
        print(f"{m:12s} {name:8s} M={M:4d}: default {base[s] * 1e6:8.1f} us {by / base[s] / 1e12:5.2f} TB/s | "
              f"tuned {t1 * 1e6:8.1f} us {by / t1 / 1e12:5.2f} TB/s", flush=True)
    print(f"total default {tot0 * 1e3:.3f} ms tuned {tot1 * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
