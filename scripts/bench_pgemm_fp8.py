"""fp8 W8A8 prefill GEMM (csrc/ops/pgemm8.hip) vs hipBLASLt's row-wise-scaled
fp8 GEMM (torch._scaled_mm) at the Llama-3-70B TP1 projection shapes and the
bench's prefill step sizes, on the same operands; per arm: time, TF/s, and
(--power) the median sclk / package power while it loops (rocm-smi, read-only).

  python scripts/bench_pgemm_fp8.py [--power] [--m 4608,5063,8192]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402

SHAPES = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="4608,5063,8192")
    ap.add_argument("--power", action="store_true")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    if a.power:
        from scripts.gemm_clock_probe import arm  # noqa: WPS433
    g = torch.Generator(device="cuda").manual_seed(0)
    tot = {"pgemm8": 0.0, "scaled_mm": 0.0}
    for M in [int(v) for v in a.m.split(",")]:
        x = torch.randn(M, 8192 * 4, generator=g, device="cuda").to(torch.bfloat16)
        for name in a.shapes.split(","):
            N, K = SHAPES[name]
            xq, xs = ops.quant_fp8_rows(x[:, :K].contiguous())
            wq, ws = ops.quant_fp8_weight(torch.randn(N, K, generator=g, device="cuda") * 0.02)
            flops = 2.0 * M * N * K
            y1 = ops.pgemm_fp8(xq, xs, wq, ws)
            y2 = torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16)
            rel = ((y1.float() - y2.float()).abs().max() / y2.float().abs().max()).item()
            t1 = timeit(lambda: ops.pgemm_fp8(xq, xs, wq, ws, out=y1))
            t2 = timeit(lambda: torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16))
            yp = ops.pgemm_fp8(xq, xs, wq, ws, persistent=True)
            relp = ((yp.float() - y2.float()).abs().max() / y2.float().abs().max()).item()
            t3 = timeit(lambda: ops.pgemm_fp8(xq, xs, wq, ws, out=yp, persistent=True))
            tot["pgemm8"] += t1
            tot["scaled_mm"] += t2
            tot["persistent"] = tot.get("persistent", 0.0) + t3
            line = (f"M={M:5d} {name:8s} N={N:5d} K={K:5d}: pgemm8 {t1:8.1f} us {flops / t1 / 1e6:6.0f} TF/s | "
                    f"persistent {t3:8.1f} us {flops / t3 / 1e6:6.0f} TF/s | "
                    f"scaled_mm {t2:8.1f} us {flops / t2 / 1e6:6.0f} TF/s | speedup {t2 / min(t1, t3):5.3f} | "
                    f"max rel diff {max(rel, relp):.2e}")
            print(line, flush=True)
            if a.power:  # arm() prints: us, TF/s, sclk, package power, TF/s per GHz
                arm(f"  pgemm8 M={M} {name}", lambda: ops.pgemm_fp8(xq, xs, wq, ws, out=y1), flops, secs=3.0)
                arm(f"  scaled_mm M={M} {name}", lambda: torch._scaled_mm(
                    xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16), flops, secs=3.0)
            del wq, ws, y1, y2
    print(f"total: pgemm8 {tot['pgemm8']:.0f} us, persistent {tot.get('persistent', 0):.0f} us, "
          f"scaled_mm {tot['scaled_mm']:.0f} us", flush=True)


if __name__ == "__main__":
    main()
