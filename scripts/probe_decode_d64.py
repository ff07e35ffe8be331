"""Paged decode at head dim 64 (gpt-oss: 64 q / 8 kv heads) against head dim 128 (Llama-3-70B) at the
same KV bytes, and a sweep of the split-K count at D = 64 (the planner's pick vs alternatives).
  python scripts/probe_decode_d64.py"""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def run(B, ctx, D, Hq=64, Hkv=8, bs=64, splits=(None,)):
    dev = "cuda"
    per = math.ceil(ctx / bs)
    nb = B * per + 1
    kc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
    bt = torch.randperm(nb - 1, device=dev)[:B * per].view(B, per).int()
    q = torch.randn(B, Hq * D, device=dev, dtype=torch.bfloat16)
    sl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    out = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
    by = B * ctx * Hkv * D * 2 * 2
    plan = ops.decode_split_plan(ctx, B, Hkv, Hq // Hkv)
    for sp in splits:
        if sp is None:
            split = plan
        else:
            size = max(64, math.ceil(ctx / sp / 64) * 64)
            split = (size, math.ceil(ctx / size))
        fn = lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, 0, None, split=split,  # noqa: E731
                                      out=out, max_ctx=ctx)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 20
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / n
        print(f"B={B:4d} ctx={ctx} D={D:3d} split={split!s:>8} (plan {plan}): {t * 1e6:7.1f} us  "
              f"{by / t / 1e12:5.2f} TB/s", flush=True)
    del kc, vc
    torch.cuda.empty_cache()


if __name__ == "__main__":
    run(64, 5000, 128)
    run(128, 5150, 64)
    run(256, 5150, 64, splits=(None, 1, 2, 4, 8, 16))
