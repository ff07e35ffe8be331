"""Decode-sized MoE layers (< 56 rows per expert): block-fp8 experts on the 64-row weight-streaming
kernel (moe.hip) vs the 64-row persistent tiles (moe8.hip MB = 1, LLMD_MOE_FP8_T64), and MXFP4 experts
on their 64-row tiles (gpt-oss shape). Interleaved arms, best of two.
  python scripts/bench_moe_decode.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def t_it(fn, it=30):
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
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    for name, E, k, d, F, act, sizes in (("gpt-oss-120b", 128, 4, 2880, 2880, 2, (32, 64, 128, 256, 512, 1024)),
                                          ("DeepSeek-R1 EP8 rank", 32, 8, 7168, 2048, 0, (16, 32, 64, 128, 192))):
        torch.manual_seed(0)
        w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
        w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
        f1q, f1s = ops.quant_fp8_block_weight(w1)
        f2q, f2s = ops.quant_fp8_block_weight(w2)
        f1q, f2q = ops.pad_fp8_k(f1q, c128(d)), ops.pad_fp8_k(f2q, c128(F))
        mx = None
        if name.startswith("gpt-oss"):
            m1 = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(w1, c128(d)))
            m2 = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(w2, c128(F)))
            mx = (ops.mxfp4_kernel_layout(m1[0]), ops.mxfp4_scales_kernel_layout(m1[1]),
                  ops.mxfp4_kernel_layout(m2[0]), ops.mxfp4_scales_kernel_layout(m2[1]))
        wbytes = f1q.numel() + f2q.numel()
        del w1, w2
        for T in sizes:
            x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
            ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
            res = {}
            for _ in range(2):
                for arm in ("stream", "t64") + (("mxfp4",) if mx else ()):
                    ops.MOE_FP8_T64 = arm == "t64"
                    if arm == "mxfp4":
                        fn = lambda: ops.moe_experts_mxfp4(x, ids, wts, *mx, act)  # noqa: E731
                    else:
                        fn = lambda: ops.moe_experts_fp8(x, ids, wts, f1q, f1s, f2q, f2s, act)  # noqa: E731
                    res[arm] = min(res.get(arm, 1e9), t_it(fn))
            ops.MOE_FP8_T64 = False
            parts = " | ".join(f"{a} {t * 1e3:.3f} ms ({wbytes / t / 1e12:.2f} TB/s fp8-equiv)" for a, t in res.items())
            print(f"{name} T={T} ({T * k / E:.1f} rows/expert): {parts} | t64 vs stream {res['stream'] / res['t64']:.2f}x",
                  flush=True)
        del f1q, f2q, mx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
