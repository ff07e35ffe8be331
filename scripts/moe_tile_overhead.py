"""Per-tile fixed cost of the block-fp8 grouped GEMM (v4, csrc/ops/moe4.hip): time one gate/up GEMM
at gpt-oss-120b T=5120 routing (128 experts, top-4, N = 5760, 192-row tiles) and DeepSeek EP8 T=4096
routing (32 experts, top-8, N = 4096, 256-row tiles) for several K, and fit t = a + b * K-steps per
tile round: a is the prologue + epilogue + dispatch cost a persistent form could hide.
  python scripts/moe_tile_overhead.py"""
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


def run(name, T, E, k, N, tile, Ks, ver):
    dev = "cuda"
    C = ops.native()
    ids, _ = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    n = T * k
    max_p = ((n + E * (tile - 1)) + tile - 1) // tile * tile
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // tile, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sorted_ids, tile_e, offs, total, inv, tile)
    m_tiles = int((tile_e >= 0).sum().item())
    wgs = m_tiles * ((N + 255) // 256)
    rounds = wgs / 256
    pts = []
    for K in Ks:
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        xq, xs = ops._quant_groups_padded(x, K)
        wq, ws = ops.quant_fp8_block_weight(torch.randn(E, N, K, device=dev, dtype=torch.bfloat16) * 0.02)
        h = torch.empty(max_p, N // 2, dtype=torch.bfloat16, device=dev)
        t = t_it(lambda: C.moe_gemm4_fp8(xq, xs, k, sorted_ids, tile_e, wq, ws, h, 1, 2, 1.702, 7.0, False, None,
                                         tile, ver, total))
        pts.append((K // 128, t * 1e6 / rounds))
        del wq, ws
    xs_ = [p[0] for p in pts]
    ys_ = [p[1] for p in pts]
    mx, my = sum(xs_) / len(xs_), sum(ys_) / len(ys_)
    b = sum((a - mx) * (c - my) for a, c in zip(xs_, ys_)) / sum((a - mx) ** 2 for a in xs_)
    a = my - b * mx
    print(f"{name} v{ver} tile={tile} m_tiles={m_tiles} workgroups={wgs} rounds={rounds:.2f}: "
          + ", ".join(f"nk={s} {u:.1f} us/round" for s, u in pts)
          + f" | fit: {a:.1f} us fixed + {b:.2f} us per K-step (fixed = {100 * a / (a + b * 23):.0f} % of a "
          f"23-step tile)", flush=True)


if __name__ == "__main__":
    vers = [int(v) for v in os.environ.get("VERS", "4").split(",")]
    for ver in vers:
        run("gpt-oss-120b T=5120", 5120, 128, 4, 5760, 192, (640, 1280, 2944, 5888), ver)
        run("deepseek-ep8 T=4096", 4096, 32, 8, 4096, 256, (1024, 2048, 4096, 7168), ver)
