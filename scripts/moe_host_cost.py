"""Host cost of one block-fp8 MoE layer call (ops.moe_experts_fp8) at gpt-oss-120b shapes: the
enqueue time per call with the GPU kept busy, and a cProfile of 20 calls naming the Python / torch
calls that take it.
  python scripts/moe_host_cost.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    T, E, k, d, F = 2048, 128, 4, 2880, 2880
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1q, w1s = ops.quant_fp8_block_weight(torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02)
    w2q, w2s = ops.quant_fp8_block_weight(torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02)
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    b2 = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.1
    ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    f = lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, 2, b1=b1, b2=b2)  # noqa: E731
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    # enqueue cost: a long GPU op first so the launches never wait on the queue
    big = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for _ in range(30):
        big @ big
    t0 = time.perf_counter()
    for _ in range(20):
        f()
    t_host = (time.perf_counter() - t0) / 20
    torch.cuda.synchronize()
    print(f"host enqueue per moe_experts_fp8 call (T={T}): {t_host * 1e6:.0f} us", flush=True)
    pr = cProfile.Profile()
    for _ in range(30):
        big @ big
    pr.enable()
    for _ in range(20):
        f()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
