"""gpt-oss-120b MoE layer at one step size (T=5405), MXFP4 or block-fp8 experts, 5 calls: a short
program for rocprofv3 counter passes.  python scripts/mxfp4_only.py [mxfp4|fp8] [T]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "mxfp4"
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 5405
    dev = "cuda"
    E, k, d, F = 128, 4, 2880, 2880
    torch.manual_seed(0)
    w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
    if kind == "mxfp4":
        q1, s1 = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(w1, 2944))
        q2, s2 = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(w2, 2944))
        q1, q2 = ops.mxfp4_kernel_layout(q1), ops.mxfp4_kernel_layout(q2)
        s1, s2 = ops.mxfp4_scales_kernel_layout(s1), ops.mxfp4_scales_kernel_layout(s2)
        fn = ops.moe_experts_mxfp4
    else:
        q1, s1 = ops.quant_fp8_block_weight(w1)
        q2, s2 = ops.quant_fp8_block_weight(w2)
        q1, q2 = ops.pad_fp8_k(q1, 2944), ops.pad_fp8_k(q2, 2944)
        fn = ops.moe_experts_fp8
    del w1, w2
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    for _ in range(5):
        fn(x, ids, wts, q1, s1, q2, s2, 2)
    torch.cuda.synchronize()
    print("ok", kind, T)


if __name__ == "__main__":
    main()
