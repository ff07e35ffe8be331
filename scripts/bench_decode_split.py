"""Decode attention under a captured-graph split plan: the plan is sized for
max_model_len (32k), the batch's contexts are short (2k). Static split (what a
graph replayed with its capture-time split size does) vs the split re-sized per
step through the device-side split size (ops.paged_decode(split_dev=...)).
Llama-3-70B TP1 heads (64 q / 8 kv, D 128), block 64, bf16 KV.
  python scripts/bench_decode_split.py"""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def main():
    Hq, Hkv, D, bs, max_len = 64, 8, 128, 64, 32768
    for B in (4, 8, 16, 32, 64):
        for ctx in (2048, 8192):
            per = math.ceil(ctx / bs)
            nb = B * per + 1
            kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
            vc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
            bt = torch.randperm(nb - 1, device="cuda")[:B * per].view(B, per).int()
            q = torch.randn(B, Hq * D, device="cuda", dtype=torch.bfloat16)
            sl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
            out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
            plan = ops.decode_split_plan(max_len, B, Hkv, Hq // Hkv)
            dyn = torch.tensor([max(64, -(-ctx // (64 * plan[1])) * 64)], dtype=torch.int32, device="cuda")
            ws = (torch.empty(B * Hq * plan[1] * D, device="cuda"), torch.empty(B * Hq * plan[1] * 2, device="cuda"))
            res = []
            for sd in (None, dyn):
                fn = lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, split=plan,  # noqa: E731
                                              out=out, workspace=ws, split_dev=sd)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(50):
                    fn()
                torch.cuda.synchronize()
                res.append((time.perf_counter() - t0) / 50)
            by = B * ctx * Hkv * D * 4
            print(f"B={B:3d} ctx={ctx:5d} plan {plan}: static split {res[0] * 1e6:7.1f} us ({by / res[0] / 1e9:5.0f} GB/s)"
                  f" | per-step split {int(dyn.item()):5d}: {res[1] * 1e6:7.1f} us ({by / res[1] / 1e9:5.0f} GB/s)")


if __name__ == "__main__":
    main()
