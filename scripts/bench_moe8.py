"""Block-fp8 grouped expert GEMM: v4 (csrc/ops/moe4.hip) vs v8 (csrc/ops/moe8.hip, persistent) on the same
aligned expert tiles, per GEMM (gate/up with the fused activation, down) and for the whole
moe_experts_fp8 layer, at gpt-oss-120b (128 experts, d = F = 2880, top-4) and DeepSeek-V3 EP8
(32 local experts, d = 7168, F = 2048, top-8) prefill-sized steps. TF/s count useful rows only.
  python scripts/bench_moe8.py [--shapes gptoss,deepseek] [--tiles 192,256]"""
import argparse
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


def run(name, T, E, k, d, F, act, tiles):
    dev = "cuda"
    C = ops.native()
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    w2q, w2s = ops.quant_fp8_block_weight(w2)
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1 if act == 2 else None
    b2 = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.1 if act == 2 else None
    ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    n = T * k
    f1, f2 = 2 * n * 2 * F * d, 2 * n * d * F
    xq, xs = ops._quant_groups_padded(x, c128(d))
    for tile in tiles:
        max_p = ((n + E * (tile - 1)) + tile - 1) // tile * tile
        sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
        tile_e = torch.empty(max_p // tile, dtype=torch.int32, device=dev)
        offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
        total = torch.empty(1, dtype=torch.int32, device=dev)
        inv = torch.empty(n, dtype=torch.int32, device=dev)
        C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sorted_ids, tile_e, offs, total, inv, tile)
        h = torch.empty(max_p, F, dtype=torch.bfloat16, device=dev)
        y = torch.empty(max_p, d, dtype=torch.bfloat16, device=dev)
        hq, hs = ops._quant_groups_padded(torch.randn(max_p, F, device=dev, dtype=torch.bfloat16), c128(F))
        row = []
        for ver in (4, 8):
            g1 = t_it(lambda: C.moe_gemm4_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, h, 1, act, 1.702, 7.0, False,
                                              b1, tile, ver, total))
            g2 = t_it(lambda: C.moe_gemm4_fp8(hq, hs, 1, sorted_ids, tile_e, w2q, w2s, y, 0, 0, 0.0, 0.0, True, b2,
                                              tile, ver, total))
            ops.MOE4_TILE, ops.MOE_FP8_V8 = str(tile), ver == 8
            lay = t_it(lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1, b2=b2))
            ops.MOE_BF16_V8 = ver == 8
            b_lay = t_it(lambda: ops.moe_experts(x, ids, wts, w1, w2, act, b1=b1, b2=b2))
            row.append(f"v{ver}: bf16 layer {b_lay * 1e3:.3f} ms {(f1 + f2) / b_lay / 1e12:.0f} TF/s, fp8 gate/up {g1 * 1e3:.3f} ms {f1 / g1 / 1e12:.0f} TF/s, down {g2 * 1e3:.3f} ms "
                       f"{f2 / g2 / 1e12:.0f} TF/s, layer {lay * 1e3:.3f} ms {(f1 + f2) / lay / 1e12:.0f} TF/s")
        ops.MOE4_TILE, ops.MOE_FP8_V8, ops.MOE_BF16_V8 = "auto", True, False
        print(f"{name} T={T} tile={tile} rows/expert={n / E:.0f}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="gptoss,deepseek")
    ap.add_argument("--tiles", default="192,256")
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",")]
    if "gptoss" in a.shapes:
        for T in (2048, 5120, 8192):
            run("gpt-oss-120b", T, 128, 4, 2880, 2880, 2, tiles)
    if "deepseek" in a.shapes:
        for T in (1024, 4096):
            run("deepseek-ep8", T, 32, 8, 7168, 2048, 0, tiles)
