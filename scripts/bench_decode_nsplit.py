"""Paged decode time vs the number of KV splits (workgroup-round quantisation):
B sequences x Hkv heads x nsplit workgroups over 256 CUs at 2 per CU.
Llama-3-70B / Qwen3-32B TP1 heads (64 q / 8 kv, D 128), bf16 KV, block 64.
  python scripts/bench_decode_nsplit.py   [NSPLIT_D=64 NSPLIT_CASES=256:5200,128:5200]"""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def main():
    D = int(os.environ.get("NSPLIT_D", "128"))  # 64: gpt-oss heads (64 q / 8 kv, D 64)
    Hq, Hkv, bs = 64, 8, 64
    cases = ((48, 7416), (110, 7400), (64, 5125), (96, 5125), (32, 7400), (160, 3000), (24, 12000))
    if os.environ.get("NSPLIT_CASES"):  # "B:ctx,B:ctx"
        cases = tuple(tuple(int(v) for v in c.split(":")) for c in os.environ["NSPLIT_CASES"].split(","))
    for B, ctx in cases:
        per = math.ceil(ctx / bs)
        nb = B * per + 1
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
        bt = torch.randperm(nb - 1, device="cuda")[:B * per].view(B, per).int()
        q = torch.randn(B, Hq * D, device="cuda", dtype=torch.bfloat16)
        sl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
        cur = ops.decode_split_plan(ctx, B, Hkv, Hq // Hkv)  # the planner's choice
        line = []
        for n in (1, 2, 3, 4, 5, 6, 8):
            split = math.ceil(ctx / n / 64) * 64
            n = math.ceil(ctx / split)
            fn = lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, split=(split, n), out=out)  # noqa
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(30):
                fn()
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / 30
            by = B * ctx * Hkv * D * 4
            line.append(f"n{n}={t * 1e6:.0f}us/{by / t / 1e12:.2f}")
        print(f"B={B:3d} ctx={ctx:5d} plan={cur}: " + " ".join(line), flush=True)


if __name__ == "__main__":
    main()
