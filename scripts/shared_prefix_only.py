"""Shared-prefix decode kernels alone (for rocprofv3 PMC passes): the
optimized-baseline shape (48 sequences, 19 groups, 6016-token prefix + 1400
own tokens, 64 q / 8 kv heads, D 128, bf16 KV, block 16), LDS-DMA variant."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
from bench_shared_prefix import tables  # noqa: E402
from llmd_amd import ops  # noqa: E402


def main():
    B, groups, P, S, Hq, Hkv, D, bs = 48, 19, 6016, 1400, 64, 8, 128, 16
    L = P + S
    rng = np.random.default_rng(0)
    bt_np, nb = tables(B, groups, P, S, bs, True, "shuffled", rng)
    kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    bt = torch.from_numpy(bt_np).cuda()
    q = torch.randn(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    sl = torch.full((B,), L, dtype=torch.int32, device="cuda")
    out = torch.empty(B, Hq * D, device="cuda", dtype=torch.bfloat16)
    plan = ops.shared_prefix_plan(bt_np, np.full(B, L, np.int32), bs, Hq // Hkv, Hkv, variant=3)
    casc = ops.cascade_tensors(plan, "cuda")
    split = ops.decode_split_plan(S, B, Hkv, Hq // Hkv)
    for _ in range(20):
        ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, split=split, out=out, cascade=casc)
    torch.cuda.synchronize()
    print("prefix bytes per call", plan.items * P * Hkv * D * 4, "suffix bytes", B * S * Hkv * D * 4)


if __name__ == "__main__":
    main()
