"""Multi-process check + microbenchmark of the symmetric IPC heap collectives
(parallel/symm.py, csrc/ops/symm.hip).

Launched with torch.distributed.run; every rank uses LLMD_SYMM_DEVICE (default
its LOCAL_RANK). With all ranks on one GPU (the 1-GPU rig) the kernels still
go through hipIpc-mapped peer memory and the per-workgroup epoch barriers.
Handles travel over gloo, so no RCCL is needed.

Checks (vs fp32 torch references):
  * custom all-reduce, one-shot and two-shot, odd sizes, in place and out of
    place, and replayed from a captured hipGraph with changing inputs;
  * EP low-latency dispatch -> expert fn -> combine with random top-k routing,
    padded rows (T < R) and a captured-graph replay;
  * fp8 dispatch (rows quantised in the dispatch kernel): received e4m3 bytes
    and scales bit-identical to ops.quant_fp8_groups of the sender's rows
    (hidden 320: a padded last group), and the block-fp8 grouped GEMM on the
    received rows vs the same experts run without EP.
Prints one JSON line per rank-0 result; exit code != 0 on any mismatch.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def expert_ref(x, ids, w, scale):
    # y_t = x_t * sum_j w_tj * (ids_tj + 1) * scale over valid ids
    f = torch.where(ids >= 0, w * (ids.float() + 1) * scale, torch.zeros_like(w)).sum(1, keepdim=True)
    return (x.float() * f)


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LLMD_SYMM_DEVICE", os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llmd_amd.parallel import symm

    bench = os.environ.get("LLMD_SYMM_BENCH", "0") == "1"
    ok = True
    res = {"world": world}
    E_local, k, d, R = 4, 4, 256, 96
    d8 = 320
    heap = symm.SymmHeap((64 << 20) + symm.SymmEP.heap_bytes(world, R, d, k)
                         + symm.SymmEP.heap_bytes(world, R, d8, k, fp8=True), rank, world)
    ar = symm.CustomAllReduce(heap, max_bytes=8 << 20, oneshot_max=256 << 10)
    sep = symm.SymmEP(heap, R, d, k)
    sep8 = symm.SymmEP(heap, R, d8, k, channel=symm.CH_EP + 1, fp8=True)

    # ---------------- all-reduce
    errs = {}
    for n in (8, 1000 * 8, 64 * 1024, 131072 + 8 * 3, 1 << 21, (8 << 20) // 2):
        xs = [torch.randn(n, generator=torch.Generator().manual_seed(100 * r + n % 97)).to(torch.bfloat16)
              for r in range(world)]
        ref = torch.stack([x.float() for x in xs]).sum(0)
        x = xs[rank].cuda()
        out = torch.empty_like(x)
        ar.all_reduce(x, out)          # out of place
        ar.all_reduce(x)               # in place
        torch.cuda.synchronize()
        e1 = (out.float().cpu() - ref).abs().max().item()
        e2 = (x.float().cpu() - ref).abs().max().item()
        tol = 0.05 * world
        errs[n] = max(e1, e2)
        if not (e1 < tol and e2 < tol):
            ok = False
            print(f"[rank {rank}] all_reduce n={n} mismatch {e1} {e2}", flush=True)
    res["allreduce_max_err"] = max(errs.values())

    # graph capture + replay with new inputs
    n = 8192 * 8
    static = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    gout = torch.empty_like(static)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.all_reduce(static, gout)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ar.all_reduce(static, gout)
    dist.barrier()
    for it in range(3):
        xs = [torch.full((n,), float(r + 1 + it), dtype=torch.bfloat16) for r in range(world)]
        static.copy_(xs[rank].cuda())
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        want = sum(r + 1 + it for r in range(world))
        if not bool((gout.float() == want).all()):
            ok = False
            print(f"[rank {rank}] graph replay {it} wrong: {gout[:4]} want {want}", flush=True)
        dist.barrier()

    # ---------------- EP dispatch / combine
    E = E_local * world
    scale = 0.01

    def expert_fn_for(p):
        def fn(rx, rid, rw):
            gid = torch.where(rid >= 0, rid + p * E_local, rid)
            return expert_ref(rx, gid, rw, scale).to(torch.bfloat16)
        return fn

    for T in (R, 37, 1):
        gen = torch.Generator().manual_seed(7 + rank * 13 + T)
        x = torch.randn(T, d, generator=gen).to(torch.bfloat16)
        ids = torch.stack([torch.randperm(E, generator=gen)[:k] for _ in range(T)]).to(torch.int32)
        if T > 3:
            ids[2, 1:] = -1  # partially routed token
        w = torch.rand(T, k, generator=gen)
        want = expert_ref(x, ids, w, scale)
        got = sep.moe(x.cuda(), ids.cuda(), w.cuda(), E_local, R, expert_fn_for(rank))
        torch.cuda.synchronize()
        err = (got.float().cpu() - want).abs().max().item()
        if not err < 0.05 + 0.02 * want.abs().max().item():
            ok = False
            print(f"[rank {rank}] ep T={T} mismatch {err}", flush=True)
        res[f"ep_err_T{T}"] = err

    # EP under graph capture
    T = 64
    sx = torch.zeros(T, d, dtype=torch.bfloat16, device="cuda")
    sids = torch.zeros(T, k, dtype=torch.int32, device="cuda")
    sw = torch.zeros(T, k, dtype=torch.float32, device="cuda")
    fn = expert_fn_for(rank)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        sep.moe(sx, sids, sw, E_local, T, fn)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        gy = sep.moe(sx, sids, sw, E_local, T, fn)
    dist.barrier()
    for it in range(3):
        gen = torch.Generator().manual_seed(1000 + rank * 7 + it)
        x = torch.randn(T, d, generator=gen).to(torch.bfloat16)
        ids = torch.stack([torch.randperm(E, generator=gen)[:k] for _ in range(T)]).to(torch.int32)
        w = torch.rand(T, k, generator=gen)
        sx.copy_(x.cuda()); sids.copy_(ids.cuda()); sw.copy_(w.cuda())
        torch.cuda.synchronize()
        dist.barrier()
        g2.replay()
        torch.cuda.synchronize()
        want = expert_ref(x, ids, w, scale)
        err = (gy.float().cpu() - want).abs().max().item()
        if not err < 0.05 + 0.02 * want.abs().max().item():
            ok = False
            print(f"[rank {rank}] ep graph replay {it} mismatch {err}", flush=True)
        dist.barrier()

    # ---------------- HT: a prefill-sized step in chunks of the heap capacity
    from llmd_amd.parallel import ep as ep_mod

    Rstep = 250
    T = Rstep - 40 * rank  # ranks hold different row counts; chunk count agreed from Rstep
    gen = torch.Generator().manual_seed(77 + rank)
    x = torch.randn(T, d, generator=gen).to(torch.bfloat16)
    ids = torch.stack([torch.randperm(E, generator=gen)[:k] for _ in range(T)]).to(torch.int32)
    w = torch.rand(T, k, generator=gen)
    got = ep_mod.symm_chunked(sep, x.cuda(), ids.cuda(), w.cuda(), E_local, Rstep, expert_fn_for(rank))
    torch.cuda.synchronize()
    want = expert_ref(x, ids, w, scale)
    err = (got.float().cpu() - want).abs().max().item()
    res["ep_ht_chunks"] = ep_mod.chunk_plan(Rstep, R)[0]
    res["ep_ht_err"] = err
    if got.shape[0] != T or not err < 0.05 + 0.02 * want.abs().max().item():
        ok = False
        print(f"[rank {rank}] ep HT chunked mismatch {err} shape {tuple(got.shape)}", flush=True)

    # ---------------- fp8 dispatch
    from llmd_amd import ops

    def inputs(src, T, dd):
        gen = torch.Generator().manual_seed(500 + src * 31 + T)
        x = (torch.randn(T, dd, generator=gen) * (1 + 4 * torch.rand(T, 1, generator=gen))).to(torch.bfloat16)
        ids = torch.stack([torch.randperm(E, generator=gen)[:k] for _ in range(T)]).to(torch.int32)
        w = torch.rand(T, k, generator=gen)
        return x, ids, w

    for T in (R, 29):
        seen = {}

        def grab(rx, rid, rw):
            seen["q"] = rx.q.view(torch.uint8).clone().cpu()
            seen["s"] = rx.s.clone().cpu()
            seen["rid"] = rid.clone().cpu()
            return torch.zeros(rx.shape[0], d8, dtype=torch.bfloat16, device="cuda")

        x, ids, w = inputs(rank, T, d8)
        sep8.moe(x.cuda(), ids.cuda(), w.cuda(), E_local, R, grab)
        torch.cuda.synchronize()
        bad = 0
        for src in range(world):
            xs_, ids_, _ = inputs(src, T, d8)
            rq, rs = ops.quant_fp8_groups(xs_.cuda())
            rq = torch.nn.functional.pad(rq.view(torch.uint8), (0, sep8.dp - d8)).cpu()
            mine = ((ids_ >= rank * E_local) & (ids_ < (rank + 1) * E_local)).any(1)
            rows = torch.arange(T)[mine] + src * R
            bad += int((seen["q"][rows] != rq[mine]).sum()) + int((seen["s"][rows] != rs.cpu()[mine]).sum())
        if bad:
            ok = False
            print(f"[rank {rank}] fp8 dispatch T={T}: {bad} bytes/scales differ from quant_fp8_groups", flush=True)
        res[f"ep_fp8_bad_T{T}"] = bad

    # real block-fp8 experts on the received rows vs no EP
    F8 = 256
    gw = torch.Generator().manual_seed(4242)
    w1 = (torch.randn(E, 2 * F8, d8, generator=gw) * 0.05).cuda()
    w2 = (torch.randn(E, d8, F8, generator=gw) * 0.05).cuda()
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    w2q, w2s = ops.quant_fp8_block_weight(w2)
    w1q = ops.pad_fp8_k(w1q, sep8.dp)
    lo = rank * E_local
    loc = (w1q[lo:lo + E_local].contiguous(), w1s[lo:lo + E_local].contiguous(),
           w2q[lo:lo + E_local].contiguous(), w2s[lo:lo + E_local].contiguous())

    def fp8_experts(rx, rid, rw):
        return ops.moe_experts_fp8(rx, rid, rw, *loc, 0)

    x, ids, w = inputs(rank, 53, d8)
    x, ids, w = x.cuda(), ids.cuda(), w.cuda()
    got = sep8.moe(x, ids, w, E_local, R, fp8_experts)
    want = ops.moe_experts_fp8(x, ids, w, w1q, w1s, w2q, w2s, 0)
    torch.cuda.synchronize()
    err = (got.float() - want.float()).abs().max().item()
    res["ep_fp8_moe_err"] = err
    if not err < 0.02 * want.float().abs().max().item() + 1e-3:
        ok = False
        print(f"[rank {rank}] fp8 EP moe mismatch {err} (max {want.float().abs().max().item()})", flush=True)

    e = heap.error()
    if e:
        ok = False
        print(f"[rank {rank}] barrier timeout flag set", flush=True)
    res["timeout_flag"] = e

    if bench:
        rows = []
        for nb in (16 << 10, 128 << 10, 512 << 10, 2 << 20, 8 << 20):
            x = torch.randn(nb // 2, device="cuda").to(torch.bfloat16)
            for _ in range(5):
                ar.all_reduce(x)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            it = 50
            for _ in range(it):
                ar.all_reduce(x)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / it * 1e6
            rows.append({"bytes": nb, "us": round(us, 1)})
            dist.barrier()
        res["allreduce_us"] = rows

    flags = torch.tensor([int(ok)])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    res["ok"] = bool(flags.item())
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    heap.close()
    dist.destroy_process_group()
    sys.exit(0 if res["ok"] else 1)


if __name__ == "__main__":
    main()
