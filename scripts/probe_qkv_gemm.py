"""Probe: hipBLASLt QKV projection of Llama-3-70B at prefill M (N = 10240 runs at
~1.0 PF/s at M = 4096 while O / gate_up / down reach 1.5-1.6, gemm_prefill_shapes.txt).
Times the fused GEMM against a weight padded to more N columns (the consumer,
rope_cache, accepts a strided [M, >= 10240] view) and a split Q | KV pair.
  python scripts/probe_qkv_gemm.py"""
import time

import torch
import torch.nn.functional as F


def t_of(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    K, N = 8192, 10240
    ws = [torch.randn(N + 2048, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(4)]  # rotate > MALL
    for M in (4096, 4608, 4672, 5120, 8192):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        i = [0]

        def nxt():
            i[0] = (i[0] + 1) % len(ws)
            return ws[i[0]]

        res = {}
        res["fused 10240"] = t_of(lambda: F.linear(x, nxt()[:N]))
        for pad in (10496, 10752, 11264, 12288):
            res[f"padded {pad}"] = t_of(lambda: F.linear(x, nxt()[:pad]))
        res["split 8192+2048"] = t_of(lambda: (F.linear(x, nxt()[:8192]), F.linear(x, nxt()[8192:N])))
        fl = 2 * M * N * K
        print(f"M={M:5d} " + " | ".join(f"{k}: {v * 1e3:.3f} ms {fl / v / 1e12:.0f} TF/s" for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
