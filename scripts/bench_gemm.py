"""Dense GEMM throughput at the Llama-3-70B TP1 prefill shapes (M tokens x
[QKV, O, gate_up, down]) through F.linear (hipBLASLt), optionally with
PyTorch TunableOp selecting among hipBLASLt/rocBLAS solutions.
  python scripts/bench_gemm.py [--tunable] [--m 8192]"""
import argparse
import os
import time

import torch
import torch.nn.functional as F


def bench(M, N, K, iters=20):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        F.linear(x, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        F.linear(x, w)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / iters
    return t, 2 * M * N * K / t / 1e12


def bench_skinny(M, N, K, iters=50):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from llmd_amd import ops

    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    res = []
    for fn in (lambda: F.linear(x, w), lambda: ops.linear(x, w)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / iters)
    by = N * K * 2
    return res, by


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tunable", action="store_true")
    ap.add_argument("--m", type=int, nargs="*", default=[8192, 4096, 64])
    ap.add_argument("--skinny", action="store_true")
    ap.add_argument("--lookup", action="store_true", help="use the repo's tuned GEMM table (what the engine runs)")
    a = ap.parse_args()
    if a.lookup:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from llmd_amd.ops.gemm_tuning import enable_lookup
        print("lookup:", enable_lookup())
    if a.skinny:
        shapes = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
                  "lm_head": (128256, 8192)}
        for M in (1, 8, 32, 64):
            tot = [0.0, 0.0]
            for name, (N, K) in shapes.items():
                (tb, ts), by = bench_skinny(M, N, K)
                tot[0] += tb
                tot[1] += ts
                print(f"M={M:3d} {name:8s}: hipBLASLt {tb * 1e6:8.1f} us {by / tb / 1e12:5.2f} TB/s | "
                      f"skinny {ts * 1e6:8.1f} us {by / ts / 1e12:5.2f} TB/s", flush=True)
            print(f"M={M:3d} layer+head total: hipBLASLt {tot[0] * 1e6:.0f} us, skinny {tot[1] * 1e6:.0f} us")
        return
    if a.tunable:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(os.path.join("gpurun_out", "tunableop_results.csv"))
    shapes = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
              "lm_head": (128256, 8192)}
    tot_t = 0.0
    for M in a.m:
        for name, (N, K) in shapes.items():
            t, tf = bench(M, N, K)
            print(f"M={M:5d} {name:8s} N={N:6d} K={K:6d}: {t * 1e3:8.3f} ms {tf:7.1f} TF/s", flush=True)
    if a.tunable:
        torch.cuda.tunable.write_file()


if __name__ == "__main__":
    main()
