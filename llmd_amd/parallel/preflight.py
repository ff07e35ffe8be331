"""Multi-GPU pre-flight for N > 1 jobs (bench.py, launch.py): prove every
cross-device path the serving topology uses works on THIS node before any
engine starts, and fail fast with a diagnostic instead of hanging inside RCCL
or silently degrading (the kvx IPC -> TCP fallback) tens of minutes later.

Checks, each collective over the job's ranks (one process per GPU):

  peer     hipDeviceCanAccessPeer for every ordered pair of the job's devices
           (xGMI peer access is what IPC / VMM mappings and the symm heap use);
  ipc      hipIpc export -> import of a neighbour's buffer + a kvx_copy_blocks
           pull of it (the kvx copy engine), compared byte for byte (the P/D KV pull);
  vmm      the chunked VMM (dmabuf fd over a Unix socket) export -> import of
           a neighbour's pool + the same pull (the decode pool's export path);
  symm_ar  the symm heap's one-shot and two-shot custom all-reduce vs RCCL
           all_reduce on integer-valued bf16 data, bit for bit (the TP path);
  ep       symm low-latency EP dispatch -> expert -> combine vs the RCCL
           all_to_all_single path of parallel/ep.py on the same routing.

Each rank reports (ok, message) per check; rank 0 prints one JSON summary.
``run`` raises PreflightError naming the failing check and ranks.
Reference: the NIXL side-channel handshake validates the peer layout before
any transfer (docs/architecture/advanced/disaggregation/operations-vllm.md:20-47);
the rdma guide's pre-deployment checks (docs/infrastructure/rdma/README.md:201-252).
"""
from __future__ import annotations

import json
import os
import socket
import struct
import tempfile
import threading
import time
import traceback
from typing import Callable, Optional

import torch
import torch.distributed as dist

CHECKS = ("peer", "ipc", "vmm", "symm_ar", "ep")


class PreflightError(RuntimeError):
    pass


def _native():
    from llmd_amd import ops

    return ops.native()


def _pattern(rank: int, n: int, device) -> torch.Tensor:
    g = torch.Generator(device="cpu").manual_seed(977 + rank)
    return torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8).to(device)


def _pull(C, dst: torch.Tensor, src_ptr: int, nbytes: int):
    pairs = torch.tensor([[0, 0]], dtype=torch.int32, device=dst.device)
    segs = torch.tensor([[0, 0, nbytes]], dtype=torch.int64, device=dst.device)
    from llmd_amd.kvx.agent import COPY_ENGINE  # the engine the P/D pulls will use

    C.kvx_copy_blocks(dst, src_ptr, nbytes, nbytes, pairs, segs, nbytes, COPY_ENGINE)
    torch.cuda.synchronize(dst.device)


def check_peer(rank, world, dev, grp, devices) -> str:
    if rank != 0:
        return "checked on rank 0"
    bad = [(a, b) for a in devices for b in devices
           if a != b and not torch.cuda.can_device_access_peer(a, b)]
    if bad:
        raise PreflightError(f"no peer access between devices {bad}")
    return f"{len(set(devices))} devices, all pairs peer-accessible"


def check_ipc(rank, world, dev, grp, devices) -> str:
    C = _native()
    n = 4 << 20
    buf = _pattern(rank, n, dev)
    h, off = C.kvx_ipc_export(buf)
    recs = [None] * world
    dist.all_gather_object(recs, (bytes(h), int(off)), group=grp)
    peer = (rank + 1) % world
    ph, poff = recs[peer]
    if peer == rank:
        return "single rank"
    base = C.kvx_ipc_open(ph)
    try:
        dst = torch.zeros(n, dtype=torch.uint8, device=dev)
        _pull(C, dst, base + poff, n)
        want = _pattern(peer, n, dev)
        if not torch.equal(dst, want):
            raise PreflightError(f"IPC pull of rank {peer}'s buffer returned wrong bytes "
                                 f"({int((dst != want).sum())} of {n} differ)")
    finally:
        dist.barrier(group=grp)  # peers keep their buffer until every importer is done
        C.kvx_ipc_close(base)
    return f"pulled 4 MiB from rank {peer} over IPC, bytes match"


def check_vmm(rank, world, dev, grp, devices) -> str:
    C = _native()
    chunk = int(C.vmm_granularity(dev.index))
    chunk = max(chunk, 2 << 20)
    pool, fds = C.vmm_pool(dev.index, chunk, 2)
    n = 2 * chunk
    pool.copy_(_pattern(rank, n, dev))
    torch.cuda.synchronize(dev)
    path = os.path.join(tempfile.gettempdir(), f"llmd-preflight-{os.getpid()}-{rank}.sock")
    if os.path.exists(path):
        os.unlink(path)
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    srv.listen(world)
    stop = threading.Event()

    def serve():
        srv.settimeout(0.2)
        while not stop.is_set():
            try:
                c, _ = srv.accept()
            except OSError:
                continue
            try:
                socket.send_fds(c, [struct.pack("<I", len(fds))], list(fds))
            finally:
                c.close()
    th = threading.Thread(target=serve, daemon=True)
    th.start()
    names = [None] * world
    dist.all_gather_object(names, path, group=grp)
    peer = (rank + 1) % world
    msg = "single rank"
    base = None
    try:
        if peer != rank:
            c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            c.settimeout(30)
            c.connect(names[peer])
            _, pfds, _, _ = socket.recv_fds(c, 16, 64)
            c.close()
            base = C.vmm_import(list(pfds), chunk, dev.index)
            for fd in pfds:
                os.close(fd)
            dst = torch.zeros(n, dtype=torch.uint8, device=dev)
            _pull(C, dst, base, n)
            want = _pattern(peer, n, dev)
            if not torch.equal(dst, want):
                raise PreflightError(f"VMM pull of rank {peer}'s pool returned wrong bytes")
            msg = f"imported rank {peer}'s 2-chunk VMM pool ({n >> 20} MiB) and pulled it, bytes match"
    finally:
        dist.barrier(group=grp)
        if base is not None:
            C.vmm_release(base)
        stop.set()
        th.join(2)
        srv.close()
        if os.path.exists(path):
            os.unlink(path)
    return msg


def check_symm_ar(rank, world, dev, grp, devices, rccl=None) -> str:
    from llmd_amd.parallel import symm

    max_bytes = 8 << 20
    slot = symm._align(max(256 << 10, max_bytes // world + 16), 256)  # CustomAllReduce's slot size
    heap = symm.SymmHeap(4 * world * slot + (2 << 20), rank, world, grp, device=dev)
    try:
        ar = symm.CustomAllReduce(heap, max_bytes=max_bytes, oneshot_max=256 << 10)
        out = []
        for n in (4096, 96 * 1024, 1 << 20, 3 * (1 << 20) + 8 * 5):  # one-shot and two-shot sizes
            g = torch.Generator(device="cpu").manual_seed(31 * rank + n)
            # small integers: every partial sum is exact in bf16, so any reduction order is bit-exact
            x = torch.randint(-8, 9, (n,), generator=g).to(torch.bfloat16).to(dev)
            got = ar.all_reduce(x, torch.empty_like(x))
            if dist.get_backend(rccl) == "gloo":  # 1-GPU rehearsal: the sum on the host (exact, integers)
                ref = x.float().cpu()
                dist.all_reduce(ref, group=rccl)
                ref = ref.to(torch.bfloat16).to(dev)
            else:
                ref = x.clone()
                dist.all_reduce(ref, group=rccl)
            torch.cuda.synchronize(dev)
            if not torch.equal(got, ref):
                raise PreflightError(f"custom all-reduce of {n} bf16 ({'one' if n * 2 <= ar.oneshot_max else 'two'}"
                                     f"-shot) differs from RCCL at {int((got != ref).sum())} elements")
            if heap.error(clear=True):
                raise PreflightError("symm barrier timed out (a peer never arrived)")
            out.append(n)
        return f"one-shot + two-shot all-reduce == RCCL bit for bit ({out})"
    finally:
        heap.close()


def check_ep(rank, world, dev, grp, devices, rccl=None) -> str:
    from llmd_amd.parallel import ep as eplib
    from llmd_amd.parallel import symm
    from llmd_amd.parallel.state import ParallelState, get_state, set_state

    E_local, k, d, T = 4, 4, 512, 48
    heap = symm.SymmHeap((8 << 20) + symm.SymmEP.heap_bytes(world, T, d, k), rank, world, grp, device=dev)
    prev = get_state()
    try:
        sep = symm.SymmEP(heap, T, d, k)
        g = torch.Generator(device="cpu").manual_seed(5 + rank)
        x = torch.randint(-4, 5, (T, d), generator=g).to(torch.bfloat16).to(dev)
        ids = torch.stack([torch.randperm(world * E_local, generator=g)[:k] for _ in range(T)]).int().to(dev)
        ids[T - 3:, 1] = -1  # some unused slots
        w = torch.randint(1, 4, (T, k), generator=g).float().to(dev)

        def expert(xr, idr, wr):  # y = x * sum_j w_j * (local id + 1): exact in bf16 for these ranges
            f = torch.where(idr >= 0, wr * (idr.float() + 1), torch.zeros_like(wr)).sum(1, keepdim=True)
            return (xr.float() * f).to(torch.bfloat16)
        got = sep.moe(x, ids, w, E_local, T, expert)
        set_state(ParallelState(world_size=world, rank=rank, local_rank=dev.index, dp_size=world, dp_rank=rank,
                                ep_group=rccl, cpu_group=grp, backend="nccl"))
        ref = eplib._alltoall(x, ids, w, E_local, expert)
        torch.cuda.synchronize(dev)
        if not torch.equal(got, ref):
            raise PreflightError(f"symm EP dispatch/combine differs from the RCCL all_to_all path "
                                 f"at {int((got != ref).sum())} elements")
        if heap.error(clear=True):
            raise PreflightError("symm EP barrier timed out (a peer never arrived)")
        return f"EP dispatch/combine ({T} tokens x top-{k} over {world * E_local} experts) == RCCL all_to_all"
    finally:
        set_state(prev)
        heap.close()


_FNS: dict[str, Callable] = {"peer": check_peer, "ipc": check_ipc, "vmm": check_vmm, "symm_ar": check_symm_ar,
                             "ep": check_ep}


def run(rank: int, world: int, device: Optional[torch.device] = None, checks=CHECKS, cpu_group=None,
        rccl_group=None, log=print, raise_on_fail: bool = True) -> dict:
    """Run the checks on every rank (collective). ``cpu_group``: gloo group for
    handle exchange (default: a new one); ``rccl_group``: the RCCL group the
    results are compared against (default: the world group)."""
    t0 = time.time()
    grp = cpu_group or dist.new_group(backend="gloo")
    dev = device or torch.device("cuda", torch.cuda.current_device())
    devices = [None] * world
    dist.all_gather_object(devices, dev.index, group=grp)
    results = {}
    for name in checks:
        fn = _FNS[name]
        t = time.time()
        try:
            kw = {"rccl": rccl_group} if name in ("symm_ar", "ep") else {}
            msg, ok = fn(rank, world, dev, grp, devices, **kw), True
        except Exception as e:  # noqa: BLE001 - reported, then raised collectively
            msg, ok = f"{type(e).__name__}: {e}", False
            log(f"[preflight rank {rank}] {name} FAILED: {msg}\n{traceback.format_exc()}")
        allr = [None] * world
        dist.all_gather_object(allr, (ok, msg), group=grp)
        bad = [r for r, (o, _) in enumerate(allr) if not o]
        results[name] = {"ok": not bad, "failed_ranks": bad, "rank0": allr[0][1],
                         "errors": {r: allr[r][1] for r in bad}, "s": round(time.time() - t, 2)}
        if bad:
            break
    summary = {"preflight": results, "world": world, "devices": devices, "s": round(time.time() - t0, 2)}
    if rank == 0:
        log("[preflight] " + json.dumps(summary))
    failed = [k for k, v in results.items() if not v["ok"]]
    if failed and raise_on_fail:
        v = results[failed[0]]
        raise PreflightError(f"pre-flight check '{failed[0]}' failed on ranks {v['failed_ranks']}: {v['errors']}")
    return summary
