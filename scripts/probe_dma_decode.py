"""Probe: plain per-sequence decode (register-staged K/V) vs routing every
sequence through the LDS-DMA shared-prefix kernel as a one-member item (its
whole context in chunks; the plain kernel gets an empty range), same outputs.
  python scripts/probe_dma_decode.py"""
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def t_of(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    Hq, Hkv, D, bs = 64, 8, 128, 64
    for B, ctx, chunk in ((64, 5125, 1024), (64, 5125, 2048), (110, 1600, 512), (110, 1600, 1024), (48, 7416, 1024),
                          (32, 8192, 1024), (128, 2000, 1024)):
        per = math.ceil(ctx / bs)
        nb = B * per + 1
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        bt = torch.randperm(nb - 1, device="cuda")[:B * per].view(B, per).int()
        q = torch.randn(B, Hq * D, device="cuda", dtype=torch.bfloat16)
        sl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
        split = ops.decode_split_plan(ctx, B, Hkv, Hq // Hkv)
        t_plain = t_of(lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, split=split, out=out))
        ref = out.clone()
        k = math.ceil(ctx / chunk)
        work = []
        for b in range(B):
            for j in range(k):
                work.append((b, 1, j * chunk, min(ctx, (j + 1) * chunk), j))
        plan = ops.SharedPrefixPlan(np.full(B, ctx, np.int32), np.full(B, k, np.int32), np.arange(B, dtype=np.int32),
                                    np.asarray(work, np.int32), B, 3, k)
        casc = ops.cascade_tensors(plan, "cuda")
        fn = lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, split=(64, 1), out=out,  # noqa
                                      cascade=casc)
        t_dma = t_of(fn)
        err = (out.float() - ref.float()).abs().max().item()
        by = B * ctx * Hkv * D * 4
        print(f"B={B:3d} ctx={ctx:5d} chunk={chunk:4d}: plain {t_plain * 1e6:7.1f} us ({by / t_plain / 1e12:.2f} TB/s) | "
              f"LDS-DMA items {t_dma * 1e6:7.1f} us ({by / t_dma / 1e12:.2f} TB/s) {len(work) * Hkv} WGs  err {err:.4f}",
              flush=True)


if __name__ == "__main__":
    main()
