"""fp8 W8A8 medium-M decode GEMM (csrc/ops/mgemm.hip F8 form) vs hipBLASLt's
row-wise-scaled fp8 GEMM (torch._scaled_mm with the TunableOp table) at a
preset's projection shapes, M 64 / 96 / 128; numerics of each winner checked
against _scaled_mm. Weights rotate through > 1 GB (cold in HBM, like decode).
Prints ROW json lines and MGEMM_FP8_TABLE entries.
  python scripts/sweep_mgemm_fp8.py --model llama-3-70b"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402
from llmd_amd.ops.gemm_tuning import enable_lookup, model_gemm_shapes  # noqa: E402

F8 = torch.float8_e4m3fn


def timed(fn, nb, iters):
    for i in range(2):
        fn(i % nb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        fn(i % nb)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--m", type=int, nargs="*", default=[64, 96, 128])
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    print("lookup:", enable_lookup())
    plans = [(w, n, s) for w in (1, 2, 4) for n in (1, 2, 3, 4, 5, 6, 8, 10) for s in (3, 4)]
    entries = []
    for name, (N, K) in model_gemm_shapes(a.model).items():
        if name == "lm_head" or K % 128:
            continue
        nb = max(2, -(-(1 << 30) // (N * K)) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.05).to(F8) for _ in range(nb)]
        wsc = (torch.rand(1, N, device="cuda") * 0.01 + 0.001).contiguous()
        for M in a.m:
            xq = torch.randn(M, K, device="cuda").to(F8)
            xs = (torch.rand(M, 1, device="cuda") * 0.01 + 0.001).contiguous()
            t_lib = timed(lambda i: torch._scaled_mm(xq, ws[i].t(), scale_a=xs, scale_b=wsc,
                                                     out_dtype=torch.bfloat16), nb, a.iters)
            best = None
            for p in plans:
                if (K // 128) < p[1]:
                    continue
                try:
                    t = timed(lambda i: ops.mgemm_fp8(xq, xs, ws[i], wsc, p), nb, a.iters)
                except RuntimeError:
                    continue
                if best is None or t < best[0]:
                    best = (t, p)
            want = torch._scaled_mm(xq, ws[0].t(), scale_a=xs, scale_b=wsc, out_dtype=torch.bfloat16).float()
            got = ops.mgemm_fp8(xq, xs, ws[0], wsc, best[1]).float()
            err = ((got - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
            ok = err < 2e-2
            by = N * K
            print(f"{a.model} {name:8s} M={M:4d}: scaled_mm {t_lib * 1e6:7.1f} us {by / t_lib / 1e12:5.2f} TB/s | "
                  f"mgemm_fp8 {best[1]} {best[0] * 1e6:7.1f} us {by / best[0] / 1e12:5.2f} TB/s | rel err {err:.2e}"
                  f"{'' if ok else ' WRONG'}", flush=True)
            print("ROW " + json.dumps({"M": M, "N": N, "K": K, "plan": best[1], "t_ours": best[0], "t_other": t_lib,
                                       "ok": ok}))
            win = ok and best[0] < 0.95 * t_lib
            entries.append(f"    ({M}, {N}, {K}): ({tuple(best[1]) if win else None}, {best[0] * 1e6:.1f}, "
                           f"{t_lib * 1e6:.1f}),")
    print("MGEMM_FP8_TABLE = {")
    print("\n".join(entries))
    print("}")


if __name__ == "__main__":
    main()
