"""Prefill GEMM (csrc/ops/pgemm.hip) vs hipBLASLt (F.linear) at the Llama-3-70B /
8B TP1 prefill shapes: correctness against an fp32 reference, then interleaved
timing rounds in one process (random uniform [-1, 1) operands, not zeros).

python scripts/bench_pgemm.py [--rounds 3] [--ms 4608,8192]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402

SHAPES = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
          "8b_qkv": (6144, 4096), "8b_gate_up": (28672, 4096), "8b_down": (4096, 14336)}


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ms", default="4608,5064,8192,2048,518")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--variants", default="0,1,2", help="pgemm variants to time (each also with split-K tail)")
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    # correctness first (small M, odd M, fused SiLU)
    for M in (1, 77, 300, 1000):
        N, K = 512, 1024
        x = torch.rand(M, K, device=dev).mul_(2).sub_(1).to(torch.bfloat16)
        w = torch.rand(N, K, device=dev).mul_(2).sub_(1).mul_(0.05).to(torch.bfloat16)
        ref = x.float() @ w.float().t()
        for v in sorted({0} | {int(t) for t in a.variants.split(",")}):
            got = ops.pgemm(x, w, variant=v).float()
            err = (got - ref).abs().max().item() / ref.abs().max().item()
            wp = ops.pgemm_pack_gate_up(w)
            g, u = ref[:, : N // 2], ref[:, N // 2:]
            sref = g * torch.sigmoid(g) * u
            sgot = (ops.pgemm_silu(x, w, variant=v) if v >= 3 else ops.pgemm(x, wp, epi=1, variant=v)).float()
            serr = (sgot - sref).abs().max().item() / sref.abs().max().item()
            print(f"check v{v} M={M} N={N} K={K}: rel err {err:.2e}  silu rel err {serr:.2e}", flush=True)
            assert err < 1e-2 and serr < 2e-2
    ms = [int(m) for m in a.ms.split(",")]
    # M = 5064: a whole 5000-token prompt beside 64 decode rows (no chunk trim)
    for M in ms:
        for name in a.shapes.split(","):
            N, K = SHAPES[name]
            x = torch.rand(M, K, device=dev).mul_(2).sub_(1).to(torch.bfloat16)
            w = torch.rand(N, K, device=dev).mul_(2).sub_(1).to(torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            flops = 2.0 * M * N * K
            it = max(3, int(2e13 / flops))
            vs = [int(v) for v in a.variants.split(",")]
            res = {"blas": []}
            for v in vs:
                res[f"v{v}"], res[f"v{v}sk"] = [], []
            fused = name.endswith("gate_up")
            if fused:
                wp = ops.pgemm_pack_gate_up(w)
                ya = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                res["blas+act"] = []
                for v in vs:
                    res[f"v{v}silu"] = []
            for _ in range(a.rounds):
                res["blas"].append(timeit(lambda: F.linear(x, w), it))
                for v in vs:
                    res[f"v{v}"].append(timeit(lambda: ops.pgemm(x, w, out=y, variant=v, split_k=False), it))
                    res[f"v{v}sk"].append(timeit(lambda: ops.pgemm(x, w, out=y, variant=v), it))
                if fused:
                    res["blas+act"].append(timeit(lambda: ops.gated_act(F.linear(x, w), ops.ACT_SILU), it))
                    for v in vs:
                        res[f"v{v}silu"].append(timeit(
                            (lambda: ops.pgemm_silu(x, w, variant=v, out=ya)) if v >= 3 else
                            (lambda: ops.pgemm(x, wp, epi=1, out=ya, variant=v)), it))
            d = max((ops.pgemm(x, w, variant=v).float() - F.linear(x, w).float()).abs().max().item() for v in vs)
            line = f"M={M:5d} {name:10s} N={N:6d} K={K:6d}:"
            for k, v in res.items():
                t = sorted(v)[len(v) // 2]
                line += f"  {k} {t:.3f} ms {flops / t / 1e9:7.1f} TF/s"
            print(line + f"  max|diff| {d:.3f}", flush=True)
            del x, w, y
            if fused:
                del wp, ya


if __name__ == "__main__":
    main()
