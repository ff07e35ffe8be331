"""Run only the GQA prefill attention at ISL 5000 (Llama-3-70B heads 64/8, D 128, block 64) a
fixed number of times - the target of a rocprofv3 --pmc pass (variant: LLMD_PREFILL_V2_VARIANT).
  python scripts/attn_only.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402
from scripts.bench_attn import make_cache  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ctx = ql = 5000
    Hq, Hkv, D, bs = 64, 8, 128, 64
    kc, vc, bt = make_cache(ctx, Hkv, D, bs, "cuda")
    q = torch.randn(ql, Hq * D, device="cuda", dtype=torch.bfloat16)
    i32 = lambda v: torch.tensor([v], dtype=torch.int32, device="cuda")  # noqa: E731
    tpi = ops.prefill_tokens_per_item(Hq, Hkv, D, bs, False)
    items = torch.tensor(ops.build_prefill_items([ql], [ctx], tpi), dtype=torch.int32, device="cuda").view(-1, 2)
    out = torch.empty(ql, Hq * D, device="cuda", dtype=torch.bfloat16)
    for _ in range(iters):
        ops.paged_prefill(q, kc, vc, bt, i32(0), i32(ql), i32(ctx), Hq, Hkv, D, D ** -0.5, 0, None, items=items,
                          out=out)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
