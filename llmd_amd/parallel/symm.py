"""Symmetric IPC heap over xGMI and the collectives built on it.

Replaces what the reference gets from NVSHMEM + DeepEP + vLLM's custom
all-reduce (reference: docker/scripts/cuda/builder/
build-nvshmem.sh:115-140, guides/wide-ep-lws/modelserver/gpu/vllm/base/
decode.yaml:119 ``--all2all-backend deepep_low_latency``) with one MI355X-native
mechanism: every rank allocates an equal-size uncached device region, exports
it through hipIpc, and maps all peers' regions (one node: 8 GPUs, 7 direct
xGMI links each). Kernels (csrc/ops/symm.hip) then push 16-byte stores into
peers' receive areas and synchronise per workgroup with epoch flags - no
host round trip, no NIC, hipGraph-capturable.

* ``CustomAllReduce`` - TP all-reduce: one-shot (push to all peers, sum N
  copies locally) for latency-bound decode sizes, two-shot (reduce-scatter +
  all-gather, 2(N-1)/N of the bytes per rank) up to ``max_bytes``; RCCL above.
* ``SymmEP`` - wide-EP low-latency dispatch/combine for decode-sized steps:
  each token row is written only to the ranks owning one of its top-k experts
  (fixed [N, R] receive layout, -1 expert rows elsewhere), the local grouped
  GEMM runs on the received rows, the weighted partial outputs are pushed
  back and summed by the token's owner. With ``fp8=True`` (block-fp8 expert
  weights) the dispatch kernel quantises each row to e4m3 + per-128 scales on
  the way out (DeepEP-LL's fused fp8 dispatch, ``use_fp8``): half the bytes
  over xGMI and no quantisation pass before the grouped GEMM.

Handles are exchanged with ``all_gather_object`` over a gloo/cpu group, so the
same code runs with RCCL ranks on 8 GPUs or with several processes sharing one
GPU (the 1-GPU test rig: hipIpc between processes on one device).
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

log = logging.getLogger("llmd.symm")

CH_ALLREDUCE = 0
CH_EP = 1
# copy received EP rows out of the uncached heap before the expert GEMM (LLMD_EP_RECV_COPY=0: read in place)
RECV_COPY = os.environ.get("LLMD_EP_RECV_COPY", "1") == "1"


def _C():
    from llmd_amd import ops

    return ops.native()


class CollectiveFailure(RuntimeError):
    """A symm collective's bounded barrier wait timed out (a peer never arrived):
    every all-reduce / EP result of that step is garbage. Fatal - the engine must
    not emit a token computed from it (the role NCCL's watchdog plays for the
    reference, TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC, docker/Dockerfile.cuda:607-608)."""


_herr_word = None  # ctypes view of the process's host-mapped failure word


def _host_err_word():
    global _herr_word
    if _herr_word is None:
        import ctypes

        _herr_word = ctypes.c_uint32.from_address(_C().symm_host_err())
    return _herr_word


def host_error() -> int:
    """The host-mapped failure word: non-zero once any symm kernel of this process
    timed out in a barrier. A plain host load, no device synchronisation."""
    return 0 if _herr_word is None else int(_herr_word.value)


def clear_host_error():
    if _herr_word is not None:
        _herr_word.value = 0


def check_health(where: str = "step"):
    """Raise CollectiveFailure if a symm barrier timed out. Called by the engine
    after every step (before its tokens are emitted) and by TP followers after
    every plan; costs one host load."""
    if _herr_word is not None and _herr_word.value:
        raise CollectiveFailure(f"symm collective timed out (a peer rank stalled or died) before {where}: "
                                "all-reduce / EP results are invalid, refusing to continue")


def _align(n: int, a: int = 4096) -> int:
    return (n + a - 1) // a * a


class SymmHeap:
    """One uncached IPC region per rank, every peer's region mapped locally.

    ``regions`` are carved by the users (all-reduce, EP) in a fixed order so
    offsets agree on every rank."""

    def __init__(self, nbytes: int, rank: int, world: int, group=None, device: Optional[torch.device] = None):
        C = _C()
        if world > 8:
            raise ValueError("symm heap spans one node (<= 8 ranks)")
        self.rank, self.world = rank, world
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.nbytes = _align(nbytes)
        if self.nbytes > (4 << 30):
            raise ValueError("hipIpc imports of >4 GiB allocations hang on this stack; keep the heap <= 4 GiB")
        _host_err_word()  # every symm launch carries the failure word's address: create it first
        self.heap = C.symm_alloc(self.nbytes, self.device.index)
        handle, off = C.kvx_ipc_export(self.heap)
        recs = [None] * world
        if world > 1:
            dist.all_gather_object(recs, (bytes(handle), int(off), self.nbytes), group=group)
        else:
            recs = [(bytes(handle), int(off), self.nbytes)]
        if any(r[2] != self.nbytes for r in recs):
            raise ValueError(f"symm heap sizes differ across ranks: {[r[2] for r in recs]}")
        self.bases: list[int] = []
        self._opened: list[int] = []
        for i, (h, o, _) in enumerate(recs):
            if i == rank:
                self.bases.append(self.heap.data_ptr())
            else:
                p = C.kvx_ipc_open(h)
                self._opened.append(p)
                self.bases.append(p + o)
        self._next = C.symm_sig_bytes()

    def carve(self, nbytes: int) -> int:
        """Reserve ``nbytes`` of the data area; returns its offset (same on all ranks)."""
        off = self._next
        if off + _align(nbytes, 256) > self.nbytes:
            raise ValueError(f"symm heap exhausted: need {off + nbytes} of {self.nbytes} bytes")
        self._next = off + _align(nbytes, 256)
        return off

    def error(self, clear: bool = False) -> int:
        """Non-zero if a barrier wait timed out (a peer never arrived)."""
        e = int(_C().symm_error(self.heap, clear))
        if clear:
            clear_host_error()
        return e

    def close(self):
        C = _C()
        for p in self._opened:
            try:
                C.kvx_ipc_close(p)
            except Exception:  # pragma: no cover - teardown best effort
                pass
        self._opened.clear()


class CustomAllReduce:
    """bf16 sum over the heap's ranks (TP group = heap ranks)."""

    def __init__(self, heap: SymmHeap, max_bytes: int = 16 << 20, oneshot_max: int = 512 << 10,
                 channel: int = CH_ALLREDUCE):
        self.heap, self.ch = heap, channel
        n = heap.world
        self.max_bytes = max_bytes
        self.oneshot_max = min(oneshot_max, max_bytes)
        # one-shot needs 2 parities x N slots of the whole message; two-shot
        # 2 parities x 2 phases x N slots of 1/N of the message.
        self.slot = _align(max(self.oneshot_max, (max_bytes + n - 1) // n + 16), 256)
        self.off = heap.carve(2 * 2 * n * self.slot)

    def should_use(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = x if out is None else out
        nb = x.numel() * 2
        mode = 1 if nb <= self.oneshot_max else 2
        _C().symm_all_reduce(self.heap.bases, self.heap.rank, self.ch, mode, self.off, self.slot, x, out)
        return out


class SymmEP:
    """Low-latency wide-EP token exchange (DeepEP-LL role) for steps of at most
    ``max_rows`` tokens per rank; the caller falls back to RCCL beyond that."""

    def __init__(self, heap: SymmHeap, max_rows: int, hidden: int, topk: int, channel: int = CH_EP,
                 fp8: bool = False):
        self.heap, self.ch = heap, channel
        n = heap.world
        self.R_max, self.d, self.k = max_rows, hidden, topk
        self.fp8 = fp8
        # fp8 dispatch: e4m3 rows padded to 128 columns + one fp32 scale per group
        self.dp = (hidden + 127) // 128 * 128
        self.ng = self.dp // 128
        rx = n * max_rows * hidden * 2
        rid = n * max_rows * topk * 4
        rw = rid
        cb = rx
        rxq = n * max_rows * self.dp if fp8 else 0
        rxs = n * max_rows * self.ng * 4 if fp8 else 0
        per = (_align(rx, 256) + _align(rid, 256) + _align(rw, 256) + _align(cb, 256) + _align(rxq, 256)
               + _align(rxs, 256))
        # Single-buffered: dispatch and combine barriers interlock (a peer's
        # dispatch e+1 needs our combine-e signal, issued after our expert GEMM
        # consumed the rows), so the receive views have fixed addresses and a
        # captured decode graph can read them directly.
        base = heap.carve(per)
        o_rx = base
        o_rid = o_rx + _align(rx, 256)
        o_rw = o_rid + _align(rid, 256)
        o_cb = o_rw + _align(rw, 256)
        o_rxq = o_cb + _align(cb, 256)
        o_rxs = o_rxq + _align(rxq, 256)
        self.layout = [o_rx, o_rid, o_rw, o_cb, 0, o_rxq if fp8 else -1, o_rxs if fp8 else -1]
        if fp8:  # padding columns are never written by the kernel: zero them once
            self.heap.heap[o_rxq:o_rxq + rxq].zero_()

    @staticmethod
    def heap_bytes(world: int, max_rows: int, hidden: int, topk: int, fp8: bool = False) -> int:
        rx = world * max_rows * hidden * 2
        rid = world * max_rows * topk * 4
        extra = 0
        if fp8:
            dp = (hidden + 127) // 128 * 128
            extra = _align(world * max_rows * dp, 256) + _align(world * max_rows * (dp // 128) * 4, 256)
        return 2 * _align(rx, 256) + 2 * _align(rid, 256) + extra + 4096

    def views(self, R: int):
        """Local receive views (rows of all src ranks) for a step of R rows per rank."""
        n = self.heap.world
        h = self.heap.heap
        o_rx, o_rid, o_rw = self.layout[:3]
        rx = h[o_rx:o_rx + n * R * self.d * 2].view(torch.bfloat16).view(n * R, self.d)
        rid = h[o_rid:o_rid + n * R * self.k * 4].view(torch.int32).view(n * R, self.k)
        rw = h[o_rw:o_rw + n * R * self.k * 4].view(torch.float32).view(n * R, self.k)
        if self.fp8:
            from llmd_amd.ops import Fp8Rows

            o_q, o_s = self.layout[5], self.layout[6]
            q = h[o_q:o_q + n * R * self.dp].view(torch.float8_e4m3fn).view(n * R, self.dp)
            s = h[o_s:o_s + n * R * self.ng * 4].view(torch.float32).view(n * R, self.ng)
            rx = Fp8Rows(q, s, self.d)
        return rx, rid, rw

    def moe(self, x: torch.Tensor, ids: torch.Tensor, w: torch.Tensor, E_local: int, R: int,
            expert_fn) -> torch.Tensor:
        """x [T, d] bf16, ids [T, k] global expert ids (-1 = none), w [T, k].
        Every rank of the heap must call with the same R (rows per rank)."""
        T = x.shape[0]
        if x.shape[1] != self.d or ids.shape[1] != self.k:
            raise ValueError(f"symm EP built for d={self.d} k={self.k}, got {tuple(x.shape)} / {tuple(ids.shape)}")
        if T > R or R > self.R_max:
            raise ValueError(f"symm EP step of {T}/{R} rows exceeds max_rows {self.R_max}")
        C = _C()
        ids = ids.to(torch.int32).contiguous()
        w = w.to(torch.float32).contiguous()
        C.symm_ep_dispatch(self.heap.bases, self.heap.rank, self.ch, self.layout, x, ids, w, R, E_local, self.fp8)
        rx, rid, rw = self.views(R)
        if RECV_COPY:
            # the heap is uncached (peers' stores must be visible without flushes): the
            # grouped GEMM re-reads each row once per N-tile of its expert, so move the
            # rows into cached memory once (one streaming copy) instead of re-fetching
            # them from HBM every time
            if self.fp8:
                from llmd_amd.ops import Fp8Rows

                rx = Fp8Rows(rx.q.clone(), rx.s.clone(), rx.d)
            else:
                rx = rx.clone()
        y = expert_fn(rx, rid, rw)
        out = torch.empty_like(x)
        C.symm_ep_combine(self.heap.bases, self.heap.rank, self.ch, self.layout, y.contiguous(), ids, R, E_local,
                          out)
        return out


_heap: Optional[SymmHeap] = None
_eps: list[SymmEP] = []
_active_mb = 0  # dual-batch overlap: micro-batch m uses EP channel CH_EP + m and its own buffers


def init(rank: int, world: int, group=None, tp_allreduce: bool = False, ep_rows: int = 0, hidden: int = 0,
         topk: int = 0, ar_max_bytes: int = 16 << 20, micro_batches: int = 1, ep_fp8: bool = False) -> SymmHeap:
    """Create the process-wide heap and install the users that were asked for.
    ``micro_batches=2`` (DBO) gives each micro-batch its own EP channel/buffers;
    ``ep_fp8`` quantises dispatched rows to block-fp8 in the dispatch kernel."""
    global _heap, _eps
    n = 1 << 20
    if tp_allreduce:
        slot = _align(max(512 << 10, ar_max_bytes // max(world, 1) + 16), 256)
        n += 4 * world * slot + 4096
    if ep_rows:
        n += micro_batches * SymmEP.heap_bytes(world, ep_rows, hidden, topk, ep_fp8)
    _heap = SymmHeap(n + (1 << 20), rank, world, group)
    if tp_allreduce:
        from .comm import set_custom_allreduce

        set_custom_allreduce(CustomAllReduce(_heap, max_bytes=ar_max_bytes))
    if ep_rows:
        _eps = [SymmEP(_heap, ep_rows, hidden, topk, channel=CH_EP + m, fp8=ep_fp8) for m in range(micro_batches)]
    log.info("symm heap %.1f MiB on rank %d/%d (allreduce=%s, ep_rows=%d, fp8 dispatch=%s)", _heap.nbytes / 2**20,
             rank, world, tp_allreduce, ep_rows, ep_fp8)
    return _heap


def ep() -> Optional[SymmEP]:
    if not _eps:
        return None
    return _eps[min(_active_mb, len(_eps) - 1)]


def micro_batches() -> int:
    """Number of EP micro-batch channels installed (2 with dual-batch overlap)."""
    return len(_eps)


def set_active_mb(m: int):
    global _active_mb
    _active_mb = m


def heap() -> Optional[SymmHeap]:
    return _heap


def shutdown():
    global _heap, _eps
    from .comm import set_custom_allreduce

    set_custom_allreduce(None)
    if _heap is not None:
        _heap.close()
    _heap, _eps = None, []


def enabled_by_env() -> bool:
    return os.environ.get("LLMD_DISABLE_CUSTOM_AR", "0") != "1"
