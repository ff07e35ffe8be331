"""MLA decode: time per split size (rows x ctx), to tune ops.mla_split_plan.
  python scripts/bench_mla_split.py"""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def main():
    H, bs = 128, 64
    for rows, ctx in ((1, 4096), (8, 4096), (32, 4096), (64, 4096), (128, 4096), (8, 16384)):
        nb_per = math.ceil(ctx / bs)
        cache = torch.randn(rows * nb_per + 1, bs, 576, dtype=torch.bfloat16, device="cuda")
        bt = torch.arange(rows * nb_per, dtype=torch.int32, device="cuda").view(rows, nb_per)
        q = torch.randn(rows, H * 576, dtype=torch.bfloat16, device="cuda")
        rr = torch.arange(rows, dtype=torch.int32, device="cuda")
        ln = torch.full((rows,), ctx, dtype=torch.int32, device="cuda")
        res = []
        for split in (64, 128, 256, 512, 1024, 2048, 4096):
            if split > ctx:
                continue
            sp = (split, math.ceil(ctx / split))
            for _ in range(3):
                ops.mla_attention(q, cache, bt, rr, ln, H, 0.05, split=sp)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                ops.mla_attention(q, cache, bt, rr, ln, H, 0.05, split=sp)
            torch.cuda.synchronize()
            res.append(f"{split}:{(time.perf_counter() - t0) / 20 * 1e6:.0f}")
        plan = ops.mla_split_plan(ctx, rows, H)
        print(f"rows={rows:4d} ctx={ctx:6d} plan={plan}  us per split: {' '.join(res)}", flush=True)


if __name__ == "__main__":
    main()
