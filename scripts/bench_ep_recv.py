"""What reading EP-received rows straight from the uncached symm heap costs the
expert GEMM (parallel/symm.py RECV_COPY): DeepSeek-R1 EP8 decode shape - 8 ranks
x R rows per rank received, 32 local block-fp8 experts, hidden 7168, moe
intermediate 2048, top-8 - the grouped GEMMs run on rows that live (a) in the
uncached heap, (b) in the heap but first copied to normal memory (the copy
included in the time), (c) in normal memory (reference).

  python scripts/bench_ep_recv.py [--rows 128] [--iters 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmd_amd import ops  # noqa: E402


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=128, help="rows per source rank")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--experts", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    d, F, k = 7168, 2048, 8
    n = a.ranks * a.rows
    dev = "cuda"
    torch.manual_seed(0)
    C = ops.native()
    dp = (d + 127) // 128 * 128
    need = n * d * 2 + n * dp + n * (dp // 128) * 4 + (1 << 20)
    heap = C.symm_alloc((need + 4095) // 4096 * 4096, 0)  # the symm heap's allocator (uncached)
    x_heap = heap[:n * d * 2].view(torch.bfloat16).view(n, d)
    x_heap.copy_(torch.randn(n, d, device=dev).to(torch.bfloat16))
    x_norm = x_heap.clone()
    # the fp8 dispatch's receive rows: e4m3 [n, dp] + scales [n, dp / 128] in the heap
    q, sc = ops.quant_fp8_groups(x_norm)
    o = n * d * 2
    q_heap = heap[o:o + n * dp].view(torch.float8_e4m3fn).view(n, dp)
    q_heap.copy_(q)
    o += n * dp
    s_heap = heap[o:o + n * (dp // 128) * 4].view(torch.float32).view(n, dp // 128)
    s_heap.copy_(sc)
    # each received row is routed to k of this rank's experts (balanced EP: every row hits)
    ids = torch.stack([torch.randperm(a.experts)[:k] for _ in range(n)]).int().to(dev)
    w = torch.rand(n, k, device=dev)
    w1 = (torch.randn(a.experts, 2 * F, d, device=dev) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(a.experts, d, F, device=dev) * 0.02).to(torch.bfloat16)
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    w2q, w2s = ops.quant_fp8_block_weight(w2)

    def fp8(x):
        return ops.moe_experts_fp8(x, ids, w, w1q, w1s, w2q, w2s, 0)

    def bf16(x):
        return ops.moe_experts(x, ids, w, w1, w2, 0)

    rows = {"fp8 dispatch rows (Fp8Rows)": (fp8, lambda: ops.Fp8Rows(q_heap, s_heap, d),
                                            lambda: ops.Fp8Rows(q_heap.clone(), s_heap.clone(), d),
                                            lambda: ops.Fp8Rows(q, sc, d)),
            "bf16 rows, bf16 experts": (bf16, lambda: x_heap, lambda: x_heap.clone(), lambda: x_norm)}
    for name, (fn, in_heap, copied, normal) in rows.items():
        r_heap = timeit(lambda: fn(in_heap()), a.iters)
        r_copy = timeit(lambda: fn(copied()), a.iters)
        r_norm = timeit(lambda: fn(normal()), a.iters)
        same = torch.equal(fn(in_heap()), fn(normal()))
        print(f"{name}: {n} rows ({a.ranks} ranks x {a.rows}), {a.experts} experts top-{k}: GEMMs reading the "
              f"uncached heap {r_heap:.1f} us | copy-out + GEMMs {r_copy:.1f} us | normal memory {r_norm:.1f} us "
              f"| identical {same}", flush=True)

if __name__ == "__main__":
    main()
