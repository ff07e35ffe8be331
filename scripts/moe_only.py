"""Run the block-fp8 grouped expert GEMMs (moe_experts_fp8) a few times at one
shape, for rocprofv3 counter passes (scripts/gpu_pmc_moe.sh, gpu_pmc_moe4.sh).
  python scripts/moe_only.py [gptoss|deepseek] [fp8|bf16]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402

SHAPES = {"gptoss": (5120, 128, 4, 2880, 2880, 2), "deepseek": (4096, 32, 8, 7168, 2048, 0)}


def main():
    T, E, k, d, F, act = SHAPES[sys.argv[1] if len(sys.argv) > 1 else "gptoss"]
    dev = "cuda"
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    w1q, w1s = ops.quant_fp8_block_weight(torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02)
    w2q, w2s = ops.quant_fp8_block_weight(torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02)
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    if len(sys.argv) > 2 and sys.argv[2] == "bf16":
        w1 = (torch.randn(E, 2 * F, d, device=dev) * 0.02).to(torch.bfloat16)
        w2 = (torch.randn(E, d, F, device=dev) * 0.02).to(torch.bfloat16)
        run = lambda: ops.moe_experts(x, ids, wts, w1, w2, act)  # noqa: E731
    else:
        run = lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act)  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        run()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / n
    print(f"T={T} E={E} k={k} d={d} F={F}: {t * 1e3:.3f} ms {2 * T * k * 3 * F * d / t / 1e12:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
