"""Does a prefill GEMM on one HIP stream overlap with prefill attention (or the
elementwise kernels) on another? Times each alone and both issued together on
two streams, Llama-3-70B TP1 shapes (one micro-batch of ~4096 tokens per
stream): if together < alone-sum by a margin, a dense two-micro-batch prefill
overlap (DBO for prefill ranks) can hide attention under GEMMs.
  python scripts/overlap_probe.py"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    from llmd_amd.ops.gemm_tuning import enable_lookup

    enable_lookup()
    dev = "cuda"
    M, K = 4096, 8192
    x = torch.randn(M, K, device=dev).bfloat16()
    wg = (torch.randn(57344, K, device=dev) * 0.02).bfloat16()  # gate_up
    wd = (torch.randn(8192, 28672, device=dev) * 0.02).bfloat16()  # down
    h = torch.randn(M, 28672, device=dev).bfloat16()
    # attention: one 5000-token sequence, last 4096 query tokens against 5000 keys (70B heads)
    Hq, Hkv, D, bs, ctx, ql = 64, 8, 128, 64, 5000, 4096
    from scripts.bench_attn import make_cache

    kc, vc, bt = make_cache(ctx, Hkv, D, bs, dev)
    q = torch.randn(ql, Hq * D, device=dev).bfloat16()
    qs = torch.zeros(1, dtype=torch.int32, device=dev)
    qln = torch.tensor([ql], dtype=torch.int32, device=dev)
    cl = torch.tensor([ctx], dtype=torch.int32, device=dev)
    tpi = ops.prefill_tokens_per_item(Hq, Hkv, D, bs)
    items = torch.tensor(ops.build_prefill_items([ql], [ctx], tpi), dtype=torch.int32, device=dev).view(-1, 2)
    out = torch.empty(ql, Hq * D, device=dev, dtype=torch.bfloat16)
    act_in = torch.randn(M, 57344, device=dev).bfloat16()

    def gemm():
        F.linear(x, wg)
        F.linear(h, wd)

    def attn():
        ops.paged_prefill(q, kc, vc, bt, qs, qln, cl, Hq, Hkv, D, D ** -0.5, 0, None, items=items, out=out)

    def elem():
        ops.gated_act(act_in)

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def both(a, b):
        main = torch.cuda.current_stream()
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):
            a()
        with torch.cuda.stream(s2):
            b()
        main.wait_stream(s1)
        main.wait_stream(s2)

    for r in range(2):
        tg, ta, te = timed(gemm), timed(attn), timed(elem)
        tga = timed(lambda: both(gemm, attn))
        tge = timed(lambda: both(gemm, elem))
        print(f"round {r}: gemm {tg * 1e3:.3f} ms  attn {ta * 1e3:.3f}  act {te * 1e3:.3f} | gemm||attn "
              f"{tga * 1e3:.3f} (sum {(tg + ta) * 1e3:.3f}, hidden {(tg + ta - tga) / ta * 100:.0f} % of attn) | "
              f"gemm||act {tge * 1e3:.3f} (sum {(tg + te) * 1e3:.3f})", flush=True)


if __name__ == "__main__":
    main()
