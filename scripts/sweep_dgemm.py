"""Decode GEMM plan sweep on the GPU: for each (model shape, M) time every
(rb, nsplit, occ) plan of csrc/ops/skinny_gemm.hip with the weights rotated
through > 1 GB (cold HBM, as in a decode step), against hipBLASLt with the
repo's TunableOp table. Prints the best plan per shape and the planner's pick.
  python scripts/sweep_dgemm.py [--model llama-3-70b] [--m 16 32 64] [--quick]"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402

SHAPES = {
    "llama-3-70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)},
    "llama-3-8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)},
}


def timed(fn, ws, iters):
    for i in range(2):
        fn(ws[i % len(ws)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        fn(ws[i % len(ws)])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--m", type=int, nargs="*", default=[16, 32, 64])
    ap.add_argument("--quick", action="store_true", help="only the planner's pick and a small neighbourhood")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    from llmd_amd.ops.gemm_tuning import enable_lookup
    enable_lookup()
    nat = ops.native()
    if a.model in SHAPES:
        shapes = SHAPES[a.model]
    else:  # any preset: its dense projection shapes at TP1
        from llmd_amd.ops.gemm_tuning import model_gemm_shapes

        shapes = {k: v for k, v in model_gemm_shapes(a.model).items() if k != "lm_head"}
    for name, (N, K) in shapes.items():
        nw = max(2, -(-(1 << 30) // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(nw)]
        by = N * K * 2
        for M in a.m:
            x = torch.randn(M, K, device="cuda").bfloat16()
            tb = timed(lambda w: F.linear(x, w), ws, a.iters)
            pick = ops.skinny_plan(M, N, K)
            res = []
            cands = set()
            if a.quick:
                rb0, ns0, occ0 = pick
                for rb in range(max(1, rb0 - 2), min(8, rb0 + 2) + 1):
                    for ns in {1, max(1, ns0 - 2), ns0 - 1, ns0, ns0 + 1, ns0 + 2, 2 * ns0}:
                        for occ in (1, 2):
                            cands.add((rb, ns, occ))
            else:
                for rb in range(1, 9):
                    for ns in (1, 2, 3, 4, 5, 6, 8, 10, 12, 16):
                        for occ in (1, 2):
                            cands.add((rb, ns, occ))
            cands.add(pick)
            want = x.float() @ ws[0].float().T
            for plan in sorted(cands):
                rb, ns, occ = plan
                if ns < 1 or ns > K // 256 or not nat.skinny_supported(M, rb, occ):
                    continue
                y = ops.skinny_gemm(x, ws[0], plan)
                err = (y.float() - want).abs().max().item()
                if err > 2e-2 * max(1.0, want.abs().max().item()):
                    print(f"  WRONG {name} M={M} plan={plan} err={err}", flush=True)
                    continue
                t = timed(lambda w: ops.skinny_gemm(x, w, plan), ws, a.iters)
                res.append((t, plan))
            res.sort()
            tp = next(t for t, p in res if p == pick) if any(p == pick for _, p in res) else float("nan")
            best_t, best = res[0]
            print(f"{a.model} {name:8s} M={M:3d}: hipBLASLt {tb * 1e6:7.1f} us {by / tb / 1e12:5.2f} TB/s | "
                  f"best {best} {best_t * 1e6:7.1f} us {by / best_t / 1e12:5.2f} TB/s | "
                  f"planner {pick} {tp * 1e6:7.1f} us", flush=True)
            print("   top5:", " ".join(f"{p}:{t * 1e6:.1f}" for t, p in res[:5]), flush=True)
            print("ROW", json.dumps({"mb": (M + 15) // 16, "M": M, "N": N, "K": K, "plan": list(best),
                                     "t_ours": best_t, "t_blas": tb}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
