"""Collective bandwidth vs message size over RCCL/xGMI (SURVEY N19 nccl-tests
role): all_reduce, all_gather, reduce_scatter, all_to_all. Reports algorithm and
bus bandwidth (nccl-tests conventions).
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/coll_bench.py [--backend gloo]"""
import argparse
import os
import time

import torch
import torch.distributed as dist


def bus_factor(op, n):
    return {"all_reduce": 2 * (n - 1) / n, "all_gather": (n - 1) / n, "reduce_scatter": (n - 1) / n,
            "all_to_all": (n - 1) / n}[op]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--max-mb", type=float, default=512)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    gpu = a.backend == "nccl"
    if gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
    dist.init_process_group(a.backend)
    dev = "cuda" if gpu else "cpu"
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    size = 1 << 10
    if rank == 0:
        print(f"{'op':15s} {'bytes':>12s} {'time_us':>10s} {'algbw GB/s':>11s} {'busbw GB/s':>11s}")
    while size <= a.max_mb * (1 << 20):
        n = size // 2
        x = torch.ones(max(world, n - n % world), dtype=torch.bfloat16 if gpu else torch.float32, device=dev)
        for op in ("all_reduce", "all_gather", "reduce_scatter", "all_to_all"):
            if op == "all_reduce":
                fn = lambda: dist.all_reduce(x)  # noqa: E731
            elif op == "all_gather":
                out = torch.empty(x.numel() * world, dtype=x.dtype, device=dev)
                fn = lambda: dist.all_gather_into_tensor(out, x)  # noqa: E731
            elif op == "reduce_scatter":
                out2 = torch.empty(x.numel() // world, dtype=x.dtype, device=dev)
                fn = lambda: dist.reduce_scatter_tensor(out2, x)  # noqa: E731
            else:
                out3 = torch.empty_like(x)
                fn = lambda: dist.all_to_all_single(out3, x)  # noqa: E731
            fn()
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fn()
            sync()
            t = (time.perf_counter() - t0) / a.iters
            nbytes = x.numel() * x.element_size()
            if rank == 0:
                alg = nbytes / t / 1e9
                print(f"{op:15s} {nbytes:12d} {t * 1e6:10.1f} {alg:11.2f} {alg * bus_factor(op, world):11.2f}",
                      flush=True)
        size *= 8
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
