"""Process-group state: one process per GPU, torch.distributed over RCCL/xGMI.

Groups:
  * world    - every rank of the job
  * tp       - tensor-parallel group (consecutive ranks: TP traffic stays on the
               direct xGMI links between neighbouring GPUs of one node)
  * dp       - data-parallel replicas (same TP rank across replicas)
  * ep       - expert parallel = tp x dp flattened (wide-EP)
  * cpu      - gloo group mirroring world, for host-side control messages
  * tp_cpu   - gloo group of one TP replica: the driver rank broadcasts each
               step's plan to its TP followers (engine/tp_worker.py)
Backend "nccl" is RCCL on ROCm. On CPU-only hosts the backend is gloo.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    ep_group: Optional[object] = None
    cpu_group: Optional[object] = None
    tp_cpu_group: Optional[object] = None  # gloo: TP step-plan broadcast
    backend: str = "none"
    tp_src: Optional[int] = None  # global rank of this replica's TP driver (default dp_rank * tp_size)

    @property
    def ep_size(self) -> int:
        return self.tp_size * self.dp_size

    @property
    def ep_rank(self) -> int:
        return self.dp_rank * self.tp_size + self.tp_rank


_STATE = ParallelState()


def get_state() -> ParallelState:
    return _STATE


def env_rank_info() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init_distributed(tp_size: int = 1, backend: Optional[str] = None,
                     timeout_s: int = 600) -> ParallelState:
    """Initialise torch.distributed from the torchrun env (MASTER_ADDR/PORT, RANK,
    WORLD_SIZE) and build TP/DP/EP groups. Safe to call with WORLD_SIZE=1."""
    global _STATE
    rank, local_rank, world = env_rank_info()
    if world % tp_size:
        raise ValueError(f"world size {world} not divisible by tp {tp_size}")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    st = ParallelState(world_size=world, rank=rank, local_rank=local_rank, tp_size=tp_size,
                       tp_rank=rank % tp_size, dp_size=world // tp_size, dp_rank=rank // tp_size,
                       backend=backend if world > 1 else "none")
    if backend == "nccl" and torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", local_rank)
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        for d in range(st.dp_size):
            ranks = list(range(d * tp_size, (d + 1) * tp_size))
            g = dist.new_group(ranks) if tp_size > 1 else None
            gc = (dist.new_group(ranks, backend="gloo") if backend != "gloo" else g) if tp_size > 1 else None
            if rank in ranks:
                st.tp_group = g
                st.tp_cpu_group = gc
        for t in range(tp_size):
            ranks = list(range(t, world, tp_size))
            g = dist.new_group(ranks) if st.dp_size > 1 else None
            if rank in ranks:
                st.dp_group = g
        st.ep_group = dist.group.WORLD
        st.cpu_group = dist.new_group(backend="gloo") if backend != "gloo" else dist.group.WORLD
    _STATE = st
    return st


def set_state(st: ParallelState):
    global _STATE
    _STATE = st


def destroy():
    global _STATE
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE = ParallelState()
