"""Collective / point-to-point bandwidth microbenchmark over RCCL (xGMI) - the
SURVEY §5.1 ``coll_bench`` / ``xgmi_bw`` tools, the MI355X counterpart of the
nccl-tests / perftest images the reference ships (docker/Dockerfile.rdma-tools).

One process per GPU (torchrun); for every op and message size it times
``--iters`` back-to-back calls between device syncs and reports nccl-tests
style algorithm and bus bandwidth (busbw = algbw x 2(n-1)/n for all-reduce,
(n-1)/n for all-gather / reduce-scatter / all-to-all, 1 for send/recv):
  all_reduce   RCCL ring/tree all-reduce (TP all-reduce above the custom AR)
  all_gather   all_gather_into_tensor (vocab-parallel logits, M02)
  reduce_scatter
  all_to_all   all_to_all_single (EP dispatch/combine fallback, M04-M06)
  sendrecv     rank 0 -> rank 1 over one direct xGMI link (P/D KV pull rate
               ceiling for a single prefiller/decoder pair, M08)
Rank 0 prints one JSON line per (op, bytes). ``--device cpu`` runs the same
code over gloo (logic rehearsal; numbers meaningless).

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/bench_coll.py
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist

OPS = ("all_reduce", "all_gather", "reduce_scatter", "all_to_all", "sendrecv")


def _bus_factor(op: str, n: int) -> float:
    if op == "all_reduce":
        return 2.0 * (n - 1) / n
    if op == "sendrecv":
        return 1.0
    return (n - 1) / n


def _make(op: str, nbytes: int, n: int, dev):
    elems = max(n, nbytes // 2 // n * n)  # bf16, divisible by the world size
    x = torch.ones(elems, dtype=torch.bfloat16, device=dev)
    if op == "all_reduce":
        return lambda: dist.all_reduce(x), elems * 2
    if op == "all_gather":
        part = x[: elems // n]
        return lambda: dist.all_gather_into_tensor(x, part), elems * 2
    if op == "reduce_scatter":
        out = torch.empty(elems // n, dtype=x.dtype, device=dev)
        return lambda: dist.reduce_scatter_tensor(out, x), elems * 2
    if op == "all_to_all":
        out = torch.empty_like(x)
        return lambda: dist.all_to_all_single(out, x), elems * 2
    if op == "sendrecv":
        rank = dist.get_rank()

        def f():
            if rank == 0:
                dist.send(x, 1)
            elif rank == 1:
                dist.recv(x, 0)
        return f, elems * 2
    raise ValueError(op)


def measure(ops, sizes, iters, warmup, dev, sync, tgroup=None):
    """Per (op, size): max over ranks of the mean time of ``iters`` calls;
    ``tgroup`` (a gloo group) carries the barriers and the max-reduction."""
    n = dist.get_world_size()
    rows = []
    for op in ops:
        if op == "sendrecv" and n < 2:
            continue
        for nb in sizes:
            fn, real = _make(op, nb, n, dev)
            for _ in range(warmup):
                fn()
            sync()
            dist.barrier(group=tgroup)
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            sync()
            dt = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=tgroup)
            t = float(dt[0])
            algbw = real / t / 1e9
            rows.append({"op": op, "bytes": real, "ranks": n, "us": round(t * 1e6, 2),
                         "algbw_GBs": round(algbw, 2), "busbw_GBs": round(algbw * _bus_factor(op, n), 2)})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", nargs="*", default=list(OPS))
    ap.add_argument("--min-bytes", type=int, default=1 << 14)
    ap.add_argument("--max-bytes", type=int, default=1 << 28)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29555")
    if a.device == "cuda":
        lr = int(os.environ.get("LOCAL_RANK", 0))
        torch.cuda.set_device(lr)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", lr))
        dev, sync = torch.device("cuda", lr), torch.cuda.synchronize
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev, sync = torch.device("cpu"), (lambda: None)
    sizes = []
    b = a.min_bytes
    while b <= a.max_bytes:
        sizes.append(b)
        b *= 4
    # barriers and the timing max-reduction ride a gloo group (CPU scalars)
    tgroup = dist.new_group(backend="gloo") if a.device == "cuda" else None
    rows = measure(a.ops, sizes, a.iters, a.warmup, dev, sync, tgroup)
    if rank == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
