"""Run the medium-M decode GEMM's best plans (from sweep logs or given) on the
70B TP2-shard shapes in a loop, for rocprofv3 kernel stats (GEMM vs reduce time).
  python scripts/mgemm_prof.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402

PLANS = {  # (N, K, M): plan
    (5120, 8192, 128): (2, 5, 3), (8192, 4096, 128): (1, 2, 3), (28672, 8192, 128): (2, 1, 3),
    (8192, 14336, 128): (4, 6, 3), (5120, 8192, 64): (2, 5, 3), (8192, 14336, 64): (4, 6, 3),
}


def main():
    for (N, K, M), plan in PLANS.items():
        nw = max(2, -(-(1 << 30) // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(nw)]
        x = torch.randn(M, K, device="cuda").bfloat16()
        for i in range(40):
            ops.mgemm(x, ws[i % nw], plan)
        torch.cuda.synchronize()
        print(N, K, M, plan, "done", flush=True)
        del ws


if __name__ == "__main__":
    main()
