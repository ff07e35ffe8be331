"""Decode attention when running sequences share a cached prefix (the
optimized-baseline / shared-prefix workloads: many requests reuse one system
prompt, the prefix cache maps them onto the same physical KV blocks).

Times, at one layer's shapes (default Qwen3-32B / Llama-3-70B TP1: 64 q / 8 kv
heads, D 128, block 64):
  unique      B sequences with private blocks (no sharing)
  shared      B sequences in G groups whose first P tokens are the same
              physical blocks (batch ordered by group, or shuffled)
  cascade     the shared-prefix decomposition: every group reads its prefix
              once (all members' query heads on the MFMA N axis), members read
              only their own suffix, partials merged by log-sum-exp
              (ops.paged_decode(..., cascade=...)); checked against the plain
              kernel's output.
  python scripts/bench_shared_prefix.py [--batch 48] [--groups 19] [--prefix 6000] [--suffix 1400]
"""
import argparse
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from llmd_amd import ops  # noqa: E402


def time_it(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def tables(B, groups, P, S, bs, shared, order, rng):
    """Block tables: group g's prefix blocks are shared by its members when
    `shared`, else every sequence gets private copies."""
    pb, sb = P // bs, math.ceil(S / bs)
    nxt = 0
    gpre = []
    for _ in range(groups):
        gpre.append(list(range(nxt, nxt + pb)))
        nxt += pb
    member = np.arange(B) % groups
    if order == "sorted":
        member = np.sort(member)
    elif order == "shuffled":
        rng.shuffle(member)
    rows = []
    for b in range(B):
        if shared:
            pre = gpre[member[b]]
        else:
            pre = list(range(nxt, nxt + pb))
            nxt += pb
        suf = list(range(nxt, nxt + sb))
        nxt += sb
        rows.append(pre + suf)
    perm = rng.permutation(nxt)  # scatter blocks over the pool like a long-running cache
    return np.array([[perm[x] for x in r] for r in rows], dtype=np.int32), nxt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=48)
    ap.add_argument("--groups", type=int, default=19)
    ap.add_argument("--prefix", type=int, default=6016)
    ap.add_argument("--suffix", type=int, default=1400)
    ap.add_argument("--hq", type=int, default=64)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--bs", type=int, default=64)
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()
    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    B, Hq, Hkv, D, bs = a.batch, a.hq, a.hkv, a.d, a.bs
    P = a.prefix // bs * bs
    L = P + a.suffix
    dt = torch.float8_e4m3fn if a.fp8 else torch.bfloat16
    q = torch.randn(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    sl = torch.full((B,), L, dtype=torch.int32, device="cuda")
    out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    kv_bytes = lambda n_tok: n_tok * Hkv * D * 2 * (1 if a.fp8 else 2)  # noqa: E731
    print(f"# B={B} groups={a.groups} prefix={P} suffix={a.suffix} Hq={Hq} Hkv={Hkv} D={D} kv={str(dt)[6:]}")
    res = {}
    for name, shared, order in [("unique", False, "sorted"), ("shared sorted", True, "sorted"),
                                ("shared shuffled", True, "shuffled")]:
        bt_np, nb = tables(B, a.groups, P, a.suffix, bs, shared, order, rng)
        kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16).to(dt)
        vc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16).to(dt)
        bt = torch.from_numpy(bt_np).cuda()
        split = ops.decode_split_plan(L, B, Hkv, Hq // Hkv)
        fn = lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, 0, None, split=split,  # noqa: E731
                                      out=out, max_ctx=L)
        t = time_it(fn)
        res[name] = t
        print(f"{name:16s}: {t * 1e6:8.1f} us  {kv_bytes(B * L) / t / 1e9:6.0f} GB/s logical KV")
        ref = out.clone()
        for variant in ((1, 3) if shared and not a.fp8 else (1,) if shared else ()):
            plan = ops.shared_prefix_plan(bt_np, np.full(B, L, np.int32), bs, Hq // Hkv, Hkv, variant=variant)
            casc = ops.cascade_tensors(plan, "cuda")
            split_c = ops.decode_split_plan(int(L - plan.sstart.min()), B, Hkv, Hq // Hkv)
            fn = lambda: ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, 0, None,  # noqa: E731
                                          split=split_c, out=out, max_ctx=L, cascade=casc)
            fn()
            err = (out.float() - ref.float()).abs().max().item()
            t = time_it(fn)
            uniq = plan.items * P + B * (L - P)
            print(f"{'cascade ' + order[:4] + ' v' + str(variant):16s}: {t * 1e6:8.1f} us  {kv_bytes(uniq) / t / 1e9:6.0f} GB/s KV actually read"
                  f"  ({plan.items} prefix items, {plan.work_units} work units; max |diff| vs plain {err:.4f})")
            assert err < 0.02, err
    # lower bound of the decomposition with the plain kernel: suffixes + one prefix per group
    bt_np, nb = tables(B, a.groups, P, a.suffix, bs, False, "sorted", rng)
    kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16).to(dt)
    vc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16).to(dt)
    bt = torch.from_numpy(bt_np).cuda()
    sls = torch.full((B,), a.suffix, dtype=torch.int32, device="cuda")
    slp = torch.full((a.groups,), P, dtype=torch.int32, device="cuda")
    sp_s = ops.decode_split_plan(a.suffix, B, Hkv, Hq // Hkv)
    sp_p = ops.decode_split_plan(P, a.groups, Hkv, Hq // Hkv)
    outg = torch.empty(a.groups, Hq * D, device="cuda", dtype=torch.bfloat16)

    def two():
        ops.paged_decode(q, kc, vc, bt[:, P // bs:], sls, Hq, Hkv, D, D ** -0.5, 0, None, split=sp_s, out=out,
                         max_ctx=a.suffix)
        ops.paged_decode(q[:a.groups], kc, vc, bt[:a.groups], slp, Hq, Hkv, D, D ** -0.5, 0, None, split=sp_p,
                         out=outg, max_ctx=P)
    t = time_it(two)
    print(f"{'plain kernel x2':16s}: {t * 1e6:8.1f} us  (suffix pass B={B} + prefix pass B={a.groups}: the reads a "
          f"cascade makes, without its merge)")


if __name__ == "__main__":
    main()
