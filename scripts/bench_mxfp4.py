"""gpt-oss-120b MoE layer: block-fp8 experts (moe_experts_fp8: v8 tiles for prefill-sized steps, the
64-row streaming kernels below 64 rows per expert) vs MXFP4 experts (moe_experts_mxfp4: the persistent
tile kernel with e2m1 weights at every step size; "2st" its default 2-buffer LDS stream (the fp8
kernel's depth), "3st" 3 buffers, LLMD_MXFP4_STAGES), same routing and activations, random weights.
  python scripts/bench_mxfp4.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def t_it(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    dev = "cuda"
    E, k, d, F = 128, 4, 2880, 2880
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    b2 = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.1
    f1q, f1s = ops.quant_fp8_block_weight(w1)
    f2q, f2s = ops.quant_fp8_block_weight(w2)
    f1q, f2q = ops.pad_fp8_k(f1q, c128(d)), ops.pad_fp8_k(f2q, c128(F))
    m1q, m1s = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(w1.float(), c128(d)))
    m2q, m2s = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(w2.float(), c128(F)))
    del w1, w2
    for T in (256, 1024, 2048, 5405, 8192):
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
        tf = t_it(lambda: ops.moe_experts_fp8(x, ids, wts, f1q, f1s, f2q, f2s, 2, b1=b1, b2=b2))
        tm = {}
        for st in ("2", "3", "2", "3"):  # interleaved, best of two
            os.environ["LLMD_MXFP4_STAGES"] = st
            t = t_it(lambda: ops.moe_experts_mxfp4(x, ids, wts, m1q, m1s, m2q, m2s, 2, b1=b1, b2=b2))
            tm[st] = min(tm.get(st, 1e9), t)
        fl = 2 * T * k * 3 * F * d
        print(f"gpt-oss-120b MoE layer T={T} ({T * k / E:.0f} rows/expert): fp8 {tf * 1e3:.3f} ms "
              f"({fl / tf / 1e12:.0f} TF/s) | mxfp4 2st {tm['2'] * 1e3:.3f} ms ({fl / tm['2'] / 1e12:.0f} TF/s) | "
              f"mxfp4 3st {tm['3'] * 1e3:.3f} ms ({fl / tm['3'] / 1e12:.0f} TF/s) | "
              f"mxfp4 3st speedup {tf / tm['3']:.2f}x", flush=True)


if __name__ == "__main__":
    main()
