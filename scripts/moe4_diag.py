"""Error map of the v4 grouped GEMMs (csrc/ops/moe4.hip) against torch on the same aligned slots:
per (tile, 32-row block of the tile, 32-column block) max error, for the bf16 form in both modes and
both A-row sources. Prints the blocks whose error exceeds the tolerance.
  python scripts/moe4_diag.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def main():
    torch.manual_seed(13)
    C = ops.native()
    dev = "cuda"
    T, E, k, d, F = 1024, 8, 2, int(os.environ.get("DIAG_D", "1024")), 512
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1 = (torch.randn(E, 2 * F, d, device=dev) * d ** -0.5).to(torch.bfloat16)
    ids, _ = ops.moe_topk(torch.randn(T, E, device=dev), k, 2)
    bm = int(sys.argv[1]) if len(sys.argv) > 1 else C.moe_tile_m_prefill()
    n = T * k
    max_p = ((n + E * (bm - 1)) + bm - 1) // bm * bm
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // bm, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    C.moe_align(ids.contiguous().view(-1), E, sorted_ids, tile_e, offs, total, inv, bm)
    sid = sorted_ids.long().cpu()
    te = tile_e.long().cpu()
    print("tiles", te.tolist())
    valid = sid >= 0
    tok = torch.where(valid, sid // k, torch.zeros_like(sid))
    ex = te.repeat_interleave(bm)
    want = torch.zeros(max_p, 2 * F)
    xf, wf = x.float().cpu(), w1.float().cpu()
    for p in range(max_p):
        if valid[p]:
            want[p] = wf[ex[p]] @ xf[tok[p]]
    for name, src, slots in (("gather", x, False), ("slots", None, True)):
        xs = src if src is not None else x[tok.to(dev)].contiguous()
        y = torch.full((max_p, 2 * F), float("nan"), device=dev, dtype=torch.bfloat16)
        C.moe_gemm4(xs, k, sorted_ids, tile_e, w1, y, 0, 0, 0.0, 0.0, slots, None, bm)
        torch.cuda.synchronize()
        err = (y.float().cpu() - want).abs()
        err[~valid] = 0
        tol = 3e-2 * want.abs().max().item()
        bad = err > tol
        print(f"{name}: max err {err.max().item():.4f} tol {tol:.4f} bad {int(bad.sum())} of {int(valid.sum()) * 2 * F}")
        if bad.any():
            eb = err.view(max_p // bm, bm // 32, 32, 2 * F // 32, 32).amax(dim=(2, 4))
            for t_, rb, cb in (eb > tol).nonzero().tolist()[:4]:
                print(f"  tile {t_} (expert {int(te[t_])}) rows {32 * rb}-{32 * rb + 31} cols {32 * cb}-{32 * cb + 31} "
                      f"err {eb[t_, rb, cb].item():.3f}")
            nt_ = max_p // bm
            frac = bad.view(nt_, bm // 16, 16, -1).float().mean(dim=(2, 3))
            for t_ in range(min(nt_, 6)):
                print(f"  tile {t_} bad fraction per 16-row block:", " ".join(f"{v:.2f}" for v in frac[t_].tolist()))
            cfrac = bad.view(max_p, -1, 16).float().mean(dim=(0, 2))
            print("  bad fraction per 16-col block:", " ".join(f"{v:.2f}" for v in cfrac.tolist()[:32]))
            rows = bad.any(1).nonzero().view(-1)
            print("  bad rows (first 40):", rows[:40].tolist())
            cols = bad.any(0).nonzero().view(-1)
            print("  bad cols (first 40):", cols[:40].tolist(), "n", len(cols))

    # mode 1 (gated activation in the epilogue) with and without bias, vs torch
    b1 = (torch.randn(E, 2 * F, device=dev) * 0.1).to(torch.bfloat16)
    for bias in (None, b1):
        want_h = torch.zeros(max_p, F)
        bf = bias.float().cpu() if bias is not None else None
        for p in range(max_p):
            if valid[p]:
                h = wf[ex[p]] @ xf[tok[p]]
                if bf is not None:
                    h = h + bf[ex[p]]
                want_h[p] = torch.nn.functional.silu(h[0::2]) * h[1::2]
        hh = torch.full((max_p, F), float("nan"), device=dev, dtype=torch.bfloat16)
        C.moe_gemm4(x, k, sorted_ids, tile_e, w1, hh, 1, 0, 1.702, 7.0, False, bias, bm)
        torch.cuda.synchronize()
        err = (hh.float().cpu() - want_h).abs()
        err[~valid] = 0
        tol = 3e-2 * want_h.abs().max().item()
        bad = err > tol
        print(f"mode1 bias={bias is not None}: max err {err.max().item():.4f} tol {tol:.4f} bad {int(bad.sum())}")
        if bad.any():
            eb = err.view(max_p // bm, bm // 32, 32, F // 32, 32).amax(dim=(2, 4))
            for t_, rb, cb in (eb > tol).nonzero().tolist()[:40]:
                print(f"  tile {t_} rows {32 * rb}-{32 * rb + 31} cols {32 * cb}-{32 * cb + 31} err {eb[t_, rb, cb].item():.3f}")
    # block-fp8 form vs the v3 256-row kernel on the same quantised operands (mode 0, gathered rows)
    c128 = lambda n_: (n_ + 127) // 128 * 128  # noqa: E731
    w1q, w1s = ops.quant_fp8_block_weight(w1.float().to(torch.bfloat16))
    w1q = ops.pad_fp8_k(w1q, c128(d))
    xq, xs = ops._quant_groups_padded(x, w1q.shape[2])
    y3 = torch.zeros(max_p, 2 * F, device=dev, dtype=torch.bfloat16)
    C.moe_gemm_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, y3, 0, 0, 0.0, 0.0, False, None, bm) if bm == 256 else None
    y4 = torch.zeros(max_p, 2 * F, device=dev, dtype=torch.bfloat16)
    C.moe_gemm4_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, y4, 0, 0, 0.0, 0.0, False, None, bm)
    if bm != 256:  # the v3 kernel has 256-row tiles only: compare against torch on the dequantised operands
        xd = (xq.float() * xs.repeat_interleave(128, 1)[:, :xq.shape[1]]).cpu()
        wd = ops.dequant_fp8_block_weight(w1q, w1s).float().cpu()
        for p in range(max_p):
            if valid[p]:
                y3[p] = (wd[ex[p]][:, :xd.shape[1]] @ xd[tok[p]]).to(torch.bfloat16).to(dev)
    torch.cuda.synchronize()
    err = (y4.float() - y3.float()).abs().cpu()  # v4 vs v3 (256) or vs torch (192)
    err[~valid] = 0
    tol = 2e-2 * y3.float().abs().max().item()
    print(f"fp8 v4 (tile {bm}) vs reference: max err {err.max().item():.4f} tol {tol:.4f} bad {int((err > tol).sum())}")
    if (err > tol).any():
        eb = err.view(max_p // bm, bm // 32, 32, 2 * F // 32, 32).amax(dim=(2, 4))
        for t_, rb, cb in (eb > tol).nonzero().tolist()[:40]:
            print(f"  tile {t_} rows {32 * rb}-{32 * rb + 31} cols {32 * cb}-{32 * cb + 31} err {eb[t_, rb, cb].item():.3f}")


if __name__ == "__main__":
    main()
