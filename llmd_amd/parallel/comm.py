"""Tensor/expert-parallel collectives.

RCCL through torch.distributed for everything; a custom one-shot IPC
all-reduce (``parallel.custom_ar``) takes over latency-bound decode-size
messages when registered. All functions are no-ops at group size 1.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .state import get_state

_custom_ar = None  # set by parallel.custom_ar.install()


def set_custom_allreduce(impl):
    global _custom_ar
    _custom_ar = impl


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    st = get_state()
    if st.tp_size == 1:
        return x
    if _custom_ar is not None and _custom_ar.should_use(x):
        return _custom_ar.all_reduce(x)
    if x.is_cuda and st.backend == "gloo":  # 1-GPU multi-process rehearsal: stage on the host
        h = x.cpu()
        dist.all_reduce(h, group=st.tp_group)
        x.copy_(h)
        return x
    dist.all_reduce(x, group=st.tp_group)
    return x


def tp_all_gather(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    st = get_state()
    if st.tp_size == 1:
        return x
    dim = dim % x.dim()
    out = torch.empty((st.tp_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if x.is_cuda and st.backend == "gloo":  # 1-GPU multi-process rehearsal: stage on the host
        parts = [torch.empty(x.shape, dtype=x.dtype) for _ in range(st.tp_size)]
        dist.all_gather(parts, x.cpu(), group=st.tp_group)
        out.copy_(torch.cat(parts, 0))
    else:
        dist.all_gather_into_tensor(out, x.contiguous(), group=st.tp_group)
    out = out.view((st.tp_size,) + tuple(x.shape))
    if dim == 0:
        return out.reshape((-1,) + tuple(x.shape[1:]))
    return torch.cat(out.unbind(0), dim=dim)


def ep_all_gather(x: torch.Tensor) -> torch.Tensor:
    """[n, ...] per rank -> [world*n, ...] (all ranks must pass equal n)."""
    st = get_state()
    if st.ep_size == 1:
        return x
    out = torch.empty((st.ep_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.contiguous(), group=st.ep_group)
    return out


def ep_reduce_scatter(x: torch.Tensor) -> torch.Tensor:
    st = get_state()
    if st.ep_size == 1:
        return x
    out = torch.empty((x.shape[0] // st.ep_size,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x.contiguous(), group=st.ep_group)
    return out


def dp_all_reduce_max_int(v: int) -> int:
    """Tiny DP lock-step sync: max of an int across DP ranks."""
    st = get_state()
    if st.dp_size == 1:
        return v
    t = torch.tensor([v], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=st.cpu_group)
    return int(t.item())


def warm_tp_group(device: torch.device):
    """Create the TP communicator with a first collective outside any hipGraph
    capture (RCCL must not initialise inside a capture)."""
    st = get_state()
    if st.tp_size == 1 or st.backend != "nccl":
        return
    t = torch.zeros(64, device=device)
    dist.all_reduce(t, group=st.tp_group)
    out = torch.empty(64 * dist.get_world_size(st.tp_group), device=device)
    dist.all_gather_into_tensor(out, t, group=st.tp_group)
    torch.cuda.synchronize(device)


def tp_src_rank() -> int:
    st = get_state()
    if st.tp_src is not None:  # replica groups not laid out from rank 0 (bench_pd decode groups)
        return st.tp_src
    return st.dp_rank * st.tp_size  # TP rank 0 of this replica drives the step


def tp_broadcast_plan(plan) -> None:
    """Driver side: send one step plan (small dict of host arrays) to TP followers."""
    st = get_state()
    dist.broadcast_object_list([plan], src=tp_src_rank(), group=st.tp_cpu_group)


def tp_recv_plan():
    st = get_state()
    box = [None]
    dist.broadcast_object_list(box, src=tp_src_rank(), group=st.tp_cpu_group)
    return box[0]


def tp_min_int(v: int) -> int:
    st = get_state()
    if st.tp_size == 1:
        return v
    t = torch.tensor([v], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.tp_cpu_group)
    return int(t.item())
