"""Medium-M decode GEMM plan sweep on the GPU: for each (model shape at TP size,
M) time every (wrb, nsplit, stages) plan of csrc/ops/mgemm.hip with the weights
rotated through > 1 GB (cold HBM, as in a decode step), against hipBLASLt with
the repo's TunableOp table and the small-M stream kernel's table pick.
  python scripts/sweep_mgemm.py [--model llama-3-70b] [--tp 1] [--m 64 96 128]"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402
from llmd_amd.ops.gemm_tuning import model_gemm_shapes  # noqa: E402


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
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--m", type=int, nargs="*", default=[64, 96, 128])
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--names", nargs="*", default=["qkv", "o", "gate_up", "down"])
    a = ap.parse_args()
    from llmd_amd.ops.gemm_tuning import enable_lookup
    enable_lookup()
    shapes = model_gemm_shapes(a.model, tp=a.tp)
    for name in a.names:
        N, K = shapes[name]
        nw = max(2, -(-(1 << 30) // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(nw)]
        by = N * K * 2
        for M in a.m:
            x = torch.randn(M, K, device="cuda").bfloat16()
            tb = timed(lambda w: F.linear(x, w), ws, a.iters)
            ts = float("inf")
            sp = ops.dgemm_choice(M, N, K) if M <= 64 else None
            if sp is not None:
                ts = timed(lambda w: ops.skinny_gemm(x, w, sp), ws, a.iters)
            want = x.float() @ ws[0].float().T
            res = []
            for wrb in (1, 2, 4):
                tiles = -(-N // (64 * wrb))
                for ns in range(1, 17):
                    if ns > K // 64 or tiles * ns > 1100:
                        continue
                    for stages in (3, 4):
                        plan = (wrb, ns, stages)
                        if not ops.native().mgemm_lds(M, wrb, stages):
                            continue
                        try:
                            y = ops.mgemm(x, ws[0], plan)
                        except RuntimeError as e:
                            print(f"  skip {plan}: {e}", flush=True)
                            continue
                        err = (y.float() - want).abs().max().item()
                        if not err <= 2e-2 * max(1.0, want.abs().max().item()):
                            print(f"  WRONG {name} M={M} plan={plan} err={err}", flush=True)
                            continue
                        t = timed(lambda w: ops.mgemm(x, w, plan), ws, a.iters)
                        res.append((t, plan))
            res.sort()
            best_t, best = res[0]
            other = min(tb, ts)
            print(f"{a.model} tp{a.tp} {name:8s} M={M:3d}: hipBLASLt {tb * 1e6:7.1f} us {by / tb / 1e12:5.2f} TB/s | "
                  f"stream {ts * 1e6:7.1f} us | mgemm {best} {best_t * 1e6:7.1f} us {by / best_t / 1e12:5.2f} TB/s",
                  flush=True)
            print("   top5:", " ".join(f"{p}:{t * 1e6:.1f}" for t, p in res[:5]), flush=True)
            print("ROW", json.dumps({"M": M, "N": N, "K": K, "plan": list(best), "t_ours": best_t,
                                     "t_other": other, "t_blas": tb}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
