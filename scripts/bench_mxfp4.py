"""gpt-oss-120b MoE layer: block-fp8 experts (moe_experts_fp8: v8 tiles for prefill-sized steps, the
64-row streaming kernels below 64 rows per expert) vs MXFP4 experts (moe_experts_mxfp4: the persistent
tile kernel with e2m1 weights: 64-row tiles for decode-sized steps, 192 / 256 rows above), same
routing and activations, random weights.
  python scripts/bench_mxfp4.py [T,T,...]"""
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
    m1k, m2k = ops.mxfp4_kernel_layout(m1q), ops.mxfp4_kernel_layout(m2q)  # the layout the model stores
    m1sk, m2sk = ops.mxfp4_scales_kernel_layout(m1s), ops.mxfp4_scales_kernel_layout(m2s)
    del w1, w2
    sizes = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [64, 256, 1024, 1536, 2048, 5405]
    for T in sizes:
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
        tf = t_it(lambda: ops.moe_experts_fp8(x, ids, wts, f1q, f1s, f2q, f2s, 2, b1=b1, b2=b2))
        # arms: default (64-row tiles below MXFP4_SMALL_ROWS rows per expert, 2 workgroups per CU),
        # "1wg" = 64-row tiles at one workgroup per CU, "big" = the 192 / 256-row tiles at every size,
        # "t64" = 64-row tiles at every size, "std" = weights in the packed standard order instead of
        # K-step major (ops.mxfp4_kernel_layout)
        arms = {"dflt": ({}, None), "std": ({}, None), "big": ({}, 0), "t64": ({}, 1 << 20)}
        tm = {}
        small = ops.MXFP4_SMALL_ROWS
        for _ in range(2):  # interleaved, best of two
            for name, (env, rows) in arms.items():
                os.environ.update(env)
                ops.MXFP4_SMALL_ROWS = small if rows is None else rows
                a1, s1, a2, s2 = (m1q, m1s, m2q, m2s) if name == "std" else (m1k, m1sk, m2k, m2sk)
                t = t_it(lambda: ops.moe_experts_mxfp4(x, ids, wts, a1, s1, a2, s2, 2, b1=b1, b2=b2))
                tm[name] = min(tm.get(name, 1e9), t)
                for key in env:
                    os.environ.pop(key)
        ops.MXFP4_SMALL_ROWS = small
        fl = 2 * T * k * 3 * F * d
        arms_s = " | ".join(f"mxfp4 {n} {t * 1e3:.3f} ms ({fl / t / 1e12:.0f} TF/s)" for n, t in tm.items())
        print(f"gpt-oss-120b MoE layer T={T} ({T * k / E:.0f} rows/expert): fp8 {tf * 1e3:.3f} ms "
              f"({fl / tf / 1e12:.0f} TF/s) | {arms_s} | mxfp4 speedup {tf / tm['dflt']:.2f}x", flush=True)


if __name__ == "__main__":
    main()
