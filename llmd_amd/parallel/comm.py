"""Tensor/expert-parallel collectives.

RCCL through torch.distributed for everything; a custom one-shot IPC
all-reduce (``parallel.custom_ar``) takes over latency-bound decode-size
messages when registered. All functions are no-ops at group size 1.
"""
from __future__ import annotations

import logging
import os
import pickle

import torch
import torch.distributed as dist

from .state import get_state

log = logging.getLogger("llmd.comm")
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


# Step-plan channel driver -> TP followers. Same host (the normal case: TP spans
# the xGMI-connected GPUs of one node): the native shared-memory broadcast ring
# (csrc/runtime/shm_ring.cpp), pickled plan in, one memcpy per follower out.
# Otherwise, or for a plan larger than a slot: gloo broadcast_object_list.
# Set up lazily by the first plan, agreed by all TP ranks (MIN over the group).
_plan_ring = None      # ShmRing, or False once the group settled on gloo
_OVERFLOW = b"\x00llmd-plan-overflow"
PLAN_SLOT_BYTES = int(os.environ.get("LLMD_TP_PLAN_SLOT_BYTES", str(8 << 20)))


def _plan_channel_driver():
    global _plan_ring
    import socket
    import uuid

    st = get_state()
    ring, name = None, None
    if os.environ.get("LLMD_TP_PLAN_SHM", "1") == "1":
        try:
            from llmd_amd import _rt_loader

            name = f"/llmd-plan-{os.getpid()}-{uuid.uuid4().hex[:8]}"
            ring = _rt_loader.rt().ShmRing(name, True, st.tp_size - 1, 4, PLAN_SLOT_BYTES)
        except Exception as e:  # noqa: BLE001 - no /dev/shm: gloo
            log.warning("TP plan ring unavailable (%s); using gloo", e)
            ring = None
    dist.broadcast_object_list([{"__plan_ring__": name if ring else None, "host": socket.gethostname()}],
                               src=tp_src_rank(), group=st.tp_cpu_group)
    ok = tp_min_int(1 if ring is not None else 0)
    if ring is not None:
        ring.unlink()  # every follower has it open (or the group falls back)
    _plan_ring = ring if ok else False


def _plan_channel_follower(hello: dict):
    global _plan_ring
    import socket

    ring = None
    if hello.get("__plan_ring__") and hello.get("host") == socket.gethostname():
        try:
            from llmd_amd import _rt_loader

            ring = _rt_loader.rt().ShmRing(hello["__plan_ring__"], False)
        except Exception as e:  # noqa: BLE001
            log.warning("TP plan ring %s not attachable (%s); using gloo", hello["__plan_ring__"], e)
    ok = tp_min_int(1 if ring is not None else 0)
    _plan_ring = ring if ok else False


def tp_broadcast_plan(plan) -> None:
    """Driver side: send one step plan (small dict of host arrays) to TP followers."""
    st = get_state()
    if _plan_ring is None:
        _plan_channel_driver()
    if _plan_ring:
        data = pickle.dumps(plan, protocol=pickle.HIGHEST_PROTOCOL)
        if _plan_ring.write(data, 600.0):
            return
        _plan_ring.write(_OVERFLOW, 600.0)  # too big for a slot: this one plan over gloo
    dist.broadcast_object_list([plan], src=tp_src_rank(), group=st.tp_cpu_group)


def tp_recv_plan():
    st = get_state()
    while True:
        if _plan_ring:
            data = _plan_ring.read(st.tp_rank - 1, 0.0)
            if data != _OVERFLOW:
                return pickle.loads(data)
        box = [None]
        dist.broadcast_object_list(box, src=tp_src_rank(), group=st.tp_cpu_group)
        msg = box[0]
        if _plan_ring is None and isinstance(msg, dict) and "__plan_ring__" in msg:
            _plan_channel_follower(msg)
            continue
        return msg


def reset_plan_channel():
    """Drop the plan ring (tests / a re-initialised TP group)."""
    global _plan_ring
    if _plan_ring:
        _plan_ring.close()
    _plan_ring = None


def tp_min_int(v: int) -> int:
    st = get_state()
    if st.tp_size == 1:
        return v
    t = torch.tensor([v], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.tp_cpu_group)
    return int(t.item())
