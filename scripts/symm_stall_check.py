"""Stalled-peer injection for the symm collectives (VERDICT r4 "fail loudly").

Launched with torch.distributed.run, 2 ranks sharing one GPU (LLMD_SYMM_DEVICE,
handles over gloo, as scripts/symm_check.py). Rank 1 plays a wedged peer: it
never enters the all-reduce. Rank 0's kernel must give up after
LLMD_SYMM_TIMEOUT_S (the bounded barrier in csrc/ops/symm.hip), set the
host-mapped failure word, and ``symm.check_health`` must raise
CollectiveFailure without any device synchronisation of its own. A healthy
all-reduce beforehand must leave the word clear.

Prints one JSON line on rank 0; exit 0 only if all of that held.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


N_MORE = 16


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LLMD_SYMM_DEVICE", os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llmd_amd.parallel import symm

    heap = symm.SymmHeap(16 << 20, rank, world)
    ar = symm.CustomAllReduce(heap, max_bytes=1 << 20, oneshot_max=256 << 10)
    x = torch.full((4096,), float(rank + 1), dtype=torch.bfloat16, device="cuda")
    y = ar.all_reduce(x)
    torch.cuda.synchronize()
    healthy = float(y[0]) == sum(range(1, world + 1)) and symm.host_error() == 0
    symm.check_health("healthy all-reduce")
    dist.barrier()
    res = {"healthy_ok": healthy}
    if rank == 0:
        t0 = time.time()
        ar.all_reduce(x)                 # rank 1 never joins: the barrier must time out
        torch.cuda.synchronize()
        res["kernel_s"] = round(time.time() - t0, 2)
        # A step issues many collectives: once one barrier timed out, the rest
        # must give up at once (the err word is read inside the wait), so N
        # more stalled all-reduces cost ~0, not N x LLMD_SYMM_TIMEOUT_S.
        t0 = time.time()
        for _ in range(N_MORE):
            ar.all_reduce(x)
        torch.cuda.synchronize()
        res["n_more"] = N_MORE
        res["more_s"] = round(time.time() - t0, 2)
        res["host_word"] = symm.host_error()
        res["device_word"] = heap.error()
        try:
            symm.check_health("stalled all-reduce")
            res["raised"] = False
        except symm.CollectiveFailure as e:
            res["raised"] = True
            res["message"] = str(e)[:120]
    dist.barrier()                       # rank 1 waits here (gloo) while rank 0's kernel times out
    if rank == 0:
        ok = res["healthy_ok"] and res["raised"] and res["host_word"] == 1 and res["device_word"] == 1
        res["ok"] = ok
        print(json.dumps(res), flush=True)
        sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
