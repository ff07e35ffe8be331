"""TP step-plan channel (parallel/comm.py): the native shared-memory broadcast
ring between a TP driver and its followers on one host, its gloo fallback, and
oversize plans that overflow a ring slot. Two CPU processes over gloo."""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.timeout(180)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _plan(i, big=False):
    n = 70000 if big else 64
    return {"step": i, "tokens": np.arange(i, i + n, dtype=np.int32), "graph": i % 2 == 0,
            "sub": {"bt": np.full((4, 8), i, dtype=np.int32)}}


def _worker(rank, port, shm, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LLMD_TP_PLAN_SHM=shm,
                      LLMD_TP_PLAN_SLOT_BYTES=str(64 << 10))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from llmd_amd.parallel import comm
    from llmd_amd.parallel.state import ParallelState, set_state

    comm.PLAN_SLOT_BYTES = 64 << 10
    set_state(ParallelState(world_size=2, rank=rank, tp_size=2, tp_rank=rank, tp_cpu_group=dist.group.WORLD,
                            cpu_group=dist.group.WORLD, tp_src=0))
    n = 300
    res = {}
    try:
        if rank == 0:
            t0 = time.perf_counter()
            for i in range(n):
                comm.tp_broadcast_plan(_plan(i, big=(i == 150)))
            comm.tp_broadcast_plan({"stop": True})
            res["us_per_plan"] = (time.perf_counter() - t0) / (n + 1) * 1e6
            res["ring"] = bool(comm._plan_ring)
        else:
            bad = 0
            for i in range(n):
                p = comm.tp_recv_plan()
                want = _plan(i, big=(i == 150))
                if not (p["step"] == i and np.array_equal(p["tokens"], want["tokens"])
                        and np.array_equal(p["sub"]["bt"], want["sub"]["bt"])):
                    bad += 1
            res["bad"] = bad
            res["stop"] = comm.tp_recv_plan().get("stop")
            res["ring"] = bool(comm._plan_ring)
        dist.barrier()
    finally:
        comm.reset_plan_channel()
        torch.save(res, f"{out}.{rank}")
        dist.destroy_process_group()


@pytest.mark.parametrize("shm", ["1", "0"])
def test_plan_channel(tmp_path, shm):
    out = str(tmp_path / "plan")
    mp.spawn(_worker, args=(_free_port(), shm, out), nprocs=2, join=True)
    d = torch.load(f"{out}.0", weights_only=False)
    f = torch.load(f"{out}.1", weights_only=False)
    assert f["bad"] == 0 and f["stop"] is True
    assert d["ring"] == f["ring"] == (shm == "1")
    print(f"plan channel shm={shm}: {d['us_per_plan']:.1f} us/plan")
