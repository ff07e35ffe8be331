"""Is the gpt-oss fp8 grouped GEMM bound by how its expert weights come from HBM? Times the v4
gate/up GEMM (csrc/ops/moe4.hip) at gpt-oss-120b T=5120 with the real routing (128 experts, one
~160-row tile each: every W byte read once, from HBM, 128 B per row per K-step) against the same
launch with every tile pointed at expert 0 (W then served by L2 / MALL) and against experts stored
in a k-slab-blocked copy read through the same kernel as a [E*NT*nk] stack of contiguous 32 KB
blocks (the same bytes per step, contiguous in HBM).
  python scripts/moe_locality_probe.py"""
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
    C = ops.native()
    T, E, k, d, F = 5120, 128, 4, 2880, 2880
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(T, d, device="cuda", generator=g).bfloat16()
    ids = torch.stack([torch.randperm(E, device="cuda", generator=g)[:k] for _ in range(T)]).int()
    w1 = torch.randn(E, 2 * F, d, device="cuda", generator=g) * 0.02
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    del w1
    Kp = (d + 127) // 128 * 128
    w1q = ops.pad_fp8_k(w1q, Kp).contiguous()
    bm = 192
    n = T * k
    max_p = ((n + E * (bm - 1)) + bm - 1) // bm * bm
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device="cuda")
    tile_e = torch.empty(max_p // bm, dtype=torch.int32, device="cuda")
    offs = torch.empty(E + 1, dtype=torch.int32, device="cuda")
    total = torch.empty(1, dtype=torch.int32, device="cuda")
    inv = torch.empty(n, dtype=torch.int32, device="cuda")
    C.moe_align(ids.view(-1), E, sorted_ids, tile_e, offs, total, inv, bm)
    xq, xs = ops._quant_groups_padded(x, Kp)
    h = torch.empty(max_p, F, dtype=torch.bfloat16, device="cuda")
    flops = 2.0 * n * 2 * F * d
    wbytes = E * 2 * F * Kp

    def run(te):
        return lambda: C.moe_gemm4_fp8(xq, xs, k, sorted_ids, te, w1q, w1s, h, 1, 2, 1.702, 7.0, False, None, bm)

    t_real = t_it(run(tile_e))
    te0 = torch.where(tile_e >= 0, torch.zeros_like(tile_e), tile_e)
    t_e0 = t_it(run(te0))
    print(f"gpt-oss gate/up fp8 v4, T={T}: real routing {t_real * 1e6:.0f} us ({flops / t_real / 1e12:.0f} TF/s, "
          f"W {wbytes / t_real / 1e9:.0f} GB/s) | all tiles on expert 0 {t_e0 * 1e6:.0f} us "
          f"({flops / t_e0 / 1e12:.0f} TF/s) | ratio {t_real / t_e0:.2f}", flush=True)


if __name__ == "__main__":
    main()
