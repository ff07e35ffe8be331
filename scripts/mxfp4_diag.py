"""Diagnostic decomposition of the MXFP4 tile GEMM's K-step (csrc/ops/moe8.hip LLMD_MXFP4_DIAG): the
gpt-oss gate/up (mode 1) and down (mode 0) GEMMs at T=5405 on 192-row tiles, timed as built (0), without
fragment reads (1), without K-step DMAs (2), without both (3: MFMAs, barriers, waits, epilogue),
without the activation (4) or the weight (8) pieces of the stream.
Outputs of 1-3 are garbage by design.  python scripts/mxfp4_diag.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    C = ops.native()
    T, E, k, d, F = 5405, 128, 4, 2880, 2880
    torch.manual_seed(0)
    w1q, w1s = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(torch.randn(E, 2 * F, d, device=dev) * 0.02, 2944))
    w2q, w2s = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(torch.randn(E, d, F, device=dev) * 0.02, 2944))
    if os.environ.get("DIAG_LAYOUT", "kstep") == "kstep":
        w1q, w2q = ops.mxfp4_kernel_layout(w1q), ops.mxfp4_kernel_layout(w2q)
        w1s, w2s = ops.mxfp4_scales_kernel_layout(w1s), ops.mxfp4_scales_kernel_layout(w2s)
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    ids, _ = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    bm = 192
    n = T * k
    max_p = ((n + E * (bm - 1)) + bm - 1) // bm * bm
    sid = torch.empty(max_p, dtype=torch.int32, device=dev)
    te = torch.empty(max_p // bm, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sid, te, offs, total, inv, bm)
    xq, xs = ops._quant_groups_padded(x, 2944)
    h = torch.zeros(max_p, F, dtype=torch.bfloat16, device=dev)
    hq, hs = ops._quant_groups_padded(h, 2944)
    y = torch.empty(max_p, d, dtype=torch.bfloat16, device=dev)
    rows = int(total.item())
    for name, fn, fl in (
            ("gate/up", lambda: C.moe_gemm8_mxfp4(xq, xs, k, sid, te, w1q, w1s, h, 1, 2, 1.702, 7.0, False, None,
                                                  bm, total), 2 * rows * 2 * F * d),
            ("down", lambda: C.moe_gemm8_mxfp4(hq, hs, 1, sid, te, w2q, w2s, y, 0, 0, 0.0, 0.0, True, None, bm,
                                               total), 2 * rows * d * F)):
        res = {}
        for _ in range(2):
            for dg in ("0", "1", "2", "3", "4", "8"):
                os.environ["LLMD_MXFP4_DIAG"] = dg
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    fn()
                torch.cuda.synchronize()
                res[dg] = min(res.get(dg, 1e9), (time.perf_counter() - t0) / 20)
        os.environ.pop("LLMD_MXFP4_DIAG")
        print(f"{name} (padded rows {rows}): " + " | ".join(
            f"{lab} {res[dg] * 1e3:.3f} ms ({fl / res[dg] / 1e12:.0f} TF/s)" for dg, lab in
            (("0", "full"), ("1", "no-frag-reads"), ("2", "no-DMA"), ("3", "neither"), ("4", "no-A-DMA"),
             ("8", "no-W-DMA"))), flush=True)


if __name__ == "__main__":
    main()
