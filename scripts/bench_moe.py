"""Grouped expert GEMM microbenchmark: bf16 vs block-fp8 (moe_experts /
moe_experts_fp8) at DeepSeek-V3 EP8 shapes (32 local experts, d=7168,
F=2048, top-8) and gpt-oss-120b (128 experts, d=F=2880, top-4).
  python scripts/bench_moe.py"""
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


def run(name, T, E, k, d, F, act):
    dev = "cuda"
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    w2q, w2s = ops.quant_fp8_block_weight(w2)
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731 - K padded as quantize_fp8 stores it on the GPU
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    tb = t_it(lambda: ops.moe_experts(x, ids, wts, w1, w2, act))
    tf = t_it(lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act))
    old_v4, old_f4 = ops.MOE_BF16_V4, ops.MOE_FP8_V4
    ops.MOE_BF16_V4 = True  # the v4 bf16 grouped GEMM (csrc/ops/moe4.hip) on the same inputs
    tb4 = t_it(lambda: ops.moe_experts(x, ids, wts, w1, w2, act))
    ops.MOE_BF16_V4 = False
    tb3 = t_it(lambda: ops.moe_experts(x, ids, wts, w1, w2, act))
    ops.MOE_BF16_V4 = old_v4
    ops.MOE_BF16_V4 = old_v4
    ops.MOE4_TILE = "192"  # 192-row expert tiles forced on (auto picks them where they pad less)
    ops.MOE_BF16_V4, ops.MOE_FP8_V4 = True, True
    tb4b = t_it(lambda: ops.moe_experts(x, ids, wts, w1, w2, act))
    tf4b = t_it(lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act))
    ops.MOE4_TILE = "256"
    tb4 = t_it(lambda: ops.moe_experts(x, ids, wts, w1, w2, act))
    ops.MOE_BF16_V4 = old_v4
    ops.MOE_FP8_V4 = True  # the v4 block-fp8 grouped GEMM (moe4.hip moe_gemm4_fp8_kernel), 256-row tiles
    tf4 = t_it(lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act))
    ops.MOE_FP8_V4 = False
    tf3 = t_it(lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act))
    ops.MOE_FP8_V4 = old_f4
    ops.MOE4_TILE = "auto"
    active = min(E, T * k)
    flops = 2 * T * k * (2 * F * d + d * F)
    wbytes_bf = active * 3 * F * d * 2
    print(f"{name} T={T}: bf16 {tb * 1e3:.3f} ms ({flops / tb / 1e12:.0f} TF/s, {wbytes_bf / tb / 1e9:.0f} GB/s w) | "
          f"fp8 {tf * 1e3:.3f} ms ({flops / tf / 1e12:.0f} TF/s, {wbytes_bf / 2 / tf / 1e9:.0f} GB/s w) "
          f"speedup {tb / tf:.2f}x | bf16 v3 {tb3 * 1e3:.3f} ms ({flops / tb3 / 1e12:.0f} TF/s) "
          f"v4 {tb4 * 1e3:.3f} ms ({flops / tb4 / 1e12:.0f} TF/s) | fp8 v3 {tf3 * 1e3:.3f} ms "
          f"({flops / tf3 / 1e12:.0f} TF/s) v4 {tf4 * 1e3:.3f} ms ({flops / tf4 / 1e12:.0f} TF/s) | v4 192-row tiles: "
          f"bf16 {flops / tb4b / 1e12:.0f} fp8 {flops / tf4b / 1e12:.0f} TF/s", flush=True)


if __name__ == "__main__":
    for T in (64, 256, 4096):
        run("deepseek-ep8", T, 32, 8, 7168, 2048, 0)
    for T in (64, 128, 1024, 5120):
        run("gpt-oss-120b", T, 128, 4, 2880, 2880, 2)
