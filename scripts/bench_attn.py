"""Microbenchmark of the paged attention kernels (prefill + decode) at the
serving shapes: Llama-3-70B TP1 heads (64 q / 8 kv, D=128), block 64.

  python scripts/bench_attn.py [--ctx 5000] [--chunk 8192] [--check]

Prefill: one sequence of `ctx` tokens prefilled in one call (causal), FLOPs =
4*Hq*D*sum_q(keys visible). Decode: batch B at context `ctx`. Prints TF/s and
GB/s; --check compares against the fp32 reference on a smaller shape first.
"""
import argparse
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if "--so" in sys.argv:  # benchmark another build of the extension (A/B)
    import importlib.machinery
    import importlib.util

    so = sys.argv[sys.argv.index("--so") + 1]
    loader = importlib.machinery.ExtensionFileLoader("llmd_amd._C", so)
    spec = importlib.util.spec_from_file_location("llmd_amd._C", so, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules["llmd_amd._C"] = mod

from llmd_amd import ops  # noqa: E402
from llmd_amd.ops import reference as ref  # noqa: E402


KV_DTYPE = torch.bfloat16


def make_cache(nctx, Hkv, D, bs, dev, seqs=1):
    nb = seqs * math.ceil(nctx / bs) + 1
    kc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16).to(KV_DTYPE)
    vc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16).to(KV_DTYPE)
    per = math.ceil(nctx / bs)
    bt = torch.stack([torch.randperm(nb - 1, device=dev)[:per] for _ in range(seqs)]).int()
    return kc, vc, bt


def time_it(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def prefill(ctx, q_len, Hq, Hkv, D, bs, check=False):
    dev = "cuda"
    kc, vc, bt = make_cache(ctx, Hkv, D, bs, dev)
    q = torch.randn(q_len, Hq * D, device=dev, dtype=torch.bfloat16)
    q_start = torch.tensor([0], dtype=torch.int32, device=dev)
    ql = torch.tensor([q_len], dtype=torch.int32, device=dev)
    cl = torch.tensor([ctx], dtype=torch.int32, device=dev)
    tpi = ops.prefill_tokens_per_item(Hq, Hkv, D, bs, KV_DTYPE == torch.float8_e4m3fn)
    items = torch.tensor(ops.build_prefill_items([q_len], [ctx], tpi), dtype=torch.int32, device=dev).view(-1, 2)
    scale = D ** -0.5
    out = torch.empty(q_len, Hq * D, device=dev, dtype=torch.bfloat16)
    fn = lambda: ops.paged_prefill(q, kc, vc, bt, q_start, ql, cl, Hq, Hkv, D, scale, 0, None,  # noqa: E731
                                   items=items, out=out)
    if check:
        fn()
        r = ref.paged_prefill(q, kc, vc, bt, q_start, ql, cl, Hq, Hkv, D, scale, 0, None)
        err = (out.float() - r.float()).abs().max().item()
        print(f"  prefill check ctx={ctx} q={q_len}: max abs err {err:.4f}")
        assert err < 0.05
    t = time_it(fn)
    p0 = ctx - q_len
    vis = sum(p0 + i + 1 for i in range(q_len))
    fl = 4 * Hq * D * vis
    print(f"prefill ctx={ctx} q={q_len} Hq={Hq} Hkv={Hkv} D={D} kv={str(KV_DTYPE)[6:]}: {t * 1e3:.3f} ms  "
          f"{fl / t / 1e12:.1f} TF/s")
    return t


def decode(ctx, B, Hq, Hkv, D, bs, layers=0):
    """layers > 0: the engine's cache layout [blocks, layers, 2, Hkv, bs, D]
    (one block of every layer contiguous, for whole-block transfers) viewed at
    one layer, instead of a per-layer [blocks, Hkv, bs, D] pool."""
    dev = "cuda"
    if layers:
        per = math.ceil(ctx / bs)
        nb = B * per + 1
        big = torch.randn(nb, layers, 2, Hkv, bs, D, device=dev, dtype=torch.bfloat16).to(KV_DTYPE)
        kc, vc = big[:, layers // 2, 0], big[:, layers // 2, 1]
        bt = torch.randperm(nb - 1, device=dev)[:B * per].view(B, per).int()
    else:
        kc, vc, bt = make_cache(ctx, Hkv, D, bs, dev, seqs=B)
    q = torch.randn(B, Hq * D, device=dev, dtype=torch.bfloat16)
    sl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    out = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
    split = ops.decode_split_plan(ctx, B, Hkv, Hq // Hkv)
    fn = lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, 0, None, split=split,  # noqa: E731
                                  out=out, max_ctx=ctx)
    t = time_it(fn)
    by = B * ctx * Hkv * D * 2 * kc.element_size()
    lay = f" engine layout L={layers}" if layers else ""
    print(f"decode B={B} ctx={ctx} kv={str(KV_DTYPE)[6:]}{lay}: {t * 1e6:.1f} us  {by / t / 1e9:.0f} GB/s (KV read)")
    return t


def mla(ctx, R, H, prefill=False, bs=64):
    dev = "cuda"
    nseq = 1 if prefill else R
    per = math.ceil(ctx / bs)
    nb = nseq * per + 1
    cache = torch.randn(nb, bs, 576, device=dev, dtype=torch.bfloat16).to(KV_DTYPE)
    bt = torch.stack([torch.randperm(nb - 1, device=dev)[:per] for _ in range(nseq)]).int()
    q = torch.randn(R, H * 576, device=dev, dtype=torch.bfloat16)
    if prefill:
        rows = torch.zeros(R, dtype=torch.int32, device=dev)
        ln = torch.arange(ctx - R + 1, ctx + 1, dtype=torch.int32, device=dev)
    else:
        rows = torch.arange(R, dtype=torch.int32, device=dev)
        ln = torch.full((R,), ctx, dtype=torch.int32, device=dev)
    out = torch.empty(R, H * 512, device=dev, dtype=torch.bfloat16)
    fn = lambda: ops.mla_attention(q, cache, bt, rows, ln, H, 0.07, max_len=ctx, out=out)  # noqa: E731
    t = time_it(fn)
    keys = float(ln.sum().item())
    fl = 2 * H * keys * (576 + 512)
    by = (nseq * ctx) * 576 * cache.element_size()
    kind = "prefill" if prefill else "decode"
    print(f"mla {kind} rows={R} ctx={ctx} H={H} kv={cache.dtype}: {t * 1e3:.3f} ms  {fl / t / 1e12:.1f} TF/s  "
          f"{by / t / 1e9:.0f} GB/s latent read")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=5000)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--so", default=None)
    ap.add_argument("--mla", action="store_true")
    ap.add_argument("--mla-only", action="store_true", help="only the MLA cases")
    ap.add_argument("--rows", type=int, default=0, help="--mla-only: just this decode batch")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--decode-layout", action="store_true",
                    help="decode only: per-layer pool vs the engine's [blocks, layers, 2, ...] layout")
    a = ap.parse_args()
    global KV_DTYPE
    KV_DTYPE = torch.float8_e4m3fn if a.kv_dtype == "fp8" else torch.bfloat16
    if a.decode_layout:
        for _ in range(2):
            decode(a.ctx, 64, 64, 8, a.D, 64)
            decode(a.ctx, 64, 64, 8, a.D, 64, layers=80)
            torch.cuda.empty_cache()
        return
    if a.mla_only:
        if a.rows:
            mla(4096, a.rows, 128)
            return
        mla(4096, 64, 128)
        mla(4096, 8, 128)
        mla(4096, 2048, 128, prefill=True)
        return
    if a.check:
        prefill(700, 300, 16, 2, a.D, 64, check=True)
        prefill(600, 600, 64, 8, a.D, 64, check=True)
    prefill(a.ctx, a.ctx, 64, 8, a.D, 64)
    prefill(a.ctx, 512, 64, 8, a.D, 64)
    prefill(8192, 8192, 64, 8, a.D, 64)
    decode(a.ctx, 64, 64, 8, a.D, 64)
    decode(a.ctx, 8, 64, 8, a.D, 64)
    if a.mla:
        mla(4096, 64, 128)
        mla(4096, 8, 128)
        mla(4096, 2048, 128, prefill=True)


if __name__ == "__main__":
    main()
