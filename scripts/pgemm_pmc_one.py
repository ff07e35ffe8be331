"""One prefill GEMM shape (default Llama-3-70B qkv at M 4608) on hipBLASLt and on
the pgemm variants, a fixed number of launches each, random [-1, 1) operands -
the workload for the rocprofv3 PMC passes of scripts/gpu_pgemm_pmc.sh."""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4608)
ap.add_argument("--n", type=int, default=10240)
ap.add_argument("--k", type=int, default=8192)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--variants", default="0,2")
a = ap.parse_args()
x = torch.rand(a.m, a.k, device="cuda").mul_(2).sub_(1).to(torch.bfloat16)
w = torch.rand(a.n, a.k, device="cuda").mul_(2).sub_(1).to(torch.bfloat16)
y = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
for _ in range(a.iters):
    F.linear(x, w)
for v in (int(s) for s in a.variants.split(",")):
    for _ in range(a.iters):
        ops.pgemm(x, w, out=y, variant=v, split_k=False)
torch.cuda.synchronize()
print("done")
