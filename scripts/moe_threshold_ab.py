"""Where the tile GEMMs (v4 bf16 / v8 fp8, 192- or 256-row expert tiles) overtake the 64-row
weight-streaming kernels (moe.hip v2): whole moe_experts / moe_experts_fp8 layer time at
gpt-oss-120b and DeepSeek EP8 shapes for a range of tokens per step, with the prefill-tile
threshold (ops.MOE_V3_MIN_ROWS, rows per local expert) off and on.
  python scripts/moe_threshold_ab.py"""
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


def run(name, E, k, d, F, act, Ts):
    dev = "cuda"
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    w2q, w2s = ops.quant_fp8_block_weight(w2)
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    default = ops.MOE_V3_MIN_ROWS
    for T in Ts:
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
        res = {}
        for thr in (10 ** 9, 0):
            ops.MOE_V3_MIN_ROWS = thr
            res[thr] = (t_it(lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act)),
                        t_it(lambda: ops.moe_experts(x, ids, wts, w1, w2, act)))
        ops.MOE_V3_MIN_ROWS = default
        (f64, b64), (ft, bt) = res[10 ** 9], res[0]
        print(f"{name} T={T} rows/expert={T * k / E:.0f}: fp8 64-row {f64 * 1e3:.3f} ms, tiles {ft * 1e3:.3f} ms "
              f"({f64 / ft:.2f}x) | bf16 64-row {b64 * 1e3:.3f} ms, tiles {bt * 1e3:.3f} ms ({b64 / bt:.2f}x)",
              flush=True)


if __name__ == "__main__":
    run("gpt-oss-120b", 128, 4, 2880, 2880, 2, (512, 1024, 1536, 2048, 3072))
    run("deepseek-ep8", 32, 8, 7168, 2048, 0, (128, 256, 384, 512))
