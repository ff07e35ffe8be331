"""kvx agent: P/D KV-cache transfer (the NIXL role in
docs/architecture/advanced/disaggregation/README.md:133-178 and
operations-vllm.md).

Roles and protocol (vLLM NixlConnector-compatible ``kv_transfer_params``):
* Prefill side (``do_remote_decode``): after the prefill the request's
  blocks are *held*; the response carries
  ``{do_remote_prefill, remote_engine_id, remote_host, remote_port,
  remote_block_ids, remote_request_id, remote_tp_size, ...}``. Blocks are
  released when the decoder sends ``free`` (after its READ) or after
  ``abort_timeout`` (VLLM_NIXL_ABORT_REQUEST_TIMEOUT, default 480 s).
* Decode side (``do_remote_prefill``): a transfer worker fetches the remote
  agent's metadata once per peer over the TCP side channel (layout
  compatibility check), then pulls the blocks one-sided:
    - ``ipc``  (GPU, same node): the peer's whole KV pool is mapped once via
      a HIP IPC handle and copied with the kvx HIP kernel (xGMI peer reads;
      heterogeneous-TP head re-slicing via copy segments; the layer-major pools
      make a block 2 L pieces, so the transfer is always the copy kernel and
      "dma" is kept only as an alias of "ipc");
    - ``rccl`` (two-sided): when both engines sit in one torch.distributed
      world (``set_p2p_group``: a group made for kvx only, so transfers never
      interleave with the engines' own collectives), the decoder asks the
      prefiller to ``push`` the blocks; the prefiller's single sender thread
      gathers them into a contiguous block-major buffer on its own stream and
      ``send``s it over RCCL (xGMI between GPUs of one node, the network
      otherwise), the decoder ``recv``s into a staging buffer and scatters it
      into its pool (TP head re-slicing by wire segments). Per prefiller the
      decoder issues push + recv under one lock and the prefiller sends in
      arrival order, so every send meets its recv;
    - ``tcp``  (CPU CI / fallback): block bytes streamed over the side channel.
  Completion -> ``free`` notification to the prefiller.
Side channel: length-prefixed msgpack request/response over TCP
(VLLM_NIXL_SIDE_CHANNEL_HOST/PORT semantics; default port 5557).
Fault injection: LLMD_KVX_FAULT=drop|delay:<s>|corrupt (probability
LLMD_KVX_FAULT_P, default 1.0) for the failure-policy tests.
Concurrency (the UCCL multi-path role, SURVEY N04, on one node): pulls run on
``LLMD_KVX_WORKERS`` (default 4) transfer threads, each with its own HIP
stream, so KV from different prefillers - different xGMI links - lands in
parallel instead of queueing behind one copy; a peer's connection, metadata
and pool mapping are set up once under a lock and shared by the workers.
Multi-link striping (the UCCL multi-path role; docs/infrastructure/
rdma/README.md:36-70): on one node every GPU pair has its own xGMI link, so a
single P->D pull over the direct link uses 1 of D's 7 links. With ``relays``
(other kvx agents on the node, e.g. the other decoders) a pull of at least
``stripe_min_bytes`` is split over 1 + k paths: the direct one, and per relay
R the two-hop P->R->D path - R copies its share of blocks from P's mapped pool
into its own IPC-exported staging buffer (one kernel, P->R link), D copies them
from R's staging into its pool (R->D link), double-buffered in chunks so the two
hops overlap. The shares run concurrently, so the pull spreads over 1 + k links
(and 1 + k of P's links).
Prefiller liveness (SGLang-style heartbeat, SURVEY M13,
operations-sglang.md:93-98): the decode side pings every known prefiller
every ``LLMD_KVX_HEARTBEAT_S`` (5 s) on a fresh connection; after
``LLMD_KVX_HEARTBEAT_FAILS`` (2) consecutive misses the peer is marked dead,
its cached connection and mapping are dropped, and pulls from it fail at once
(-> kv_load_failure_policy) instead of hanging on a dead socket. A later
successful ping revives it.
Hybrid KV caches (engine/hybrid_kv.py; gpt-oss with the hybrid manager): the
sliding-window layers live in a second pool (``kv_swa``) with their own block
tables; the prefiller holds both tables (windowed entries null before the last
window), the decoder allocated the full prompt in one group and the last
window in the other, and every transport moves each pool's non-null pairs
with that pool's own segments (``pool="swa"`` on the wire).
Tensor-parallel decoders (the reference's ``D TP4`` P/D deployments,
guides/pd-disaggregation/README.md:336-460): every TP rank of a decode
replica owns a slice of the KV heads and pulls that slice itself, straight
from the prefiller's pool into its own (head re-slicing by copy segments; no
GPU writes into another GPU's memory, so no stale-L2 hazard). The driver rank
(TP rank 0, which runs the scheduler) forwards each load / cancel to its
followers through the step-plan channel (``KvxConnector.flush_tp``);
followers report completion to the driver's side channel (``tp_done``), and
the driver reports a request as loaded only once every rank has. Each rank
sends its own ``free`` with ``{rank, of}`` and the prefiller releases the
blocks after ``of`` distinct ranks have (no rank can read freed blocks).
"""
from __future__ import annotations

import logging
import os
import queue
import random
import socket
import socketserver
import struct
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Optional

import msgpack
import numpy as np
import torch

from llmd_amd.utils import markers

log = logging.getLogger("llmd.kvx")
# block-copy engine (csrc/ops/kvx_copy.hip) of P/D pulls and the offload pack / unpack: 1 =
# LDS-staged through global_load_lds (default: 8-20 % faster than the register-staged kernel on
# 16-128-block pulls, TP re-slices and slab packs of 70B blocks, profiles/kvx_copy_engine_ab_r5.txt),
# 0 = register-staged
COPY_ENGINE = int(os.environ.get("LLMD_KVX_COPY_ENGINE", "1"))


def _send(sock, obj):
    b = msgpack.packb(obj, use_bin_type=True)
    sock.sendall(struct.pack("<Q", len(b)) + b)


def _recv(sock):
    hdr = _recvn(sock, 8)
    n = struct.unpack("<Q", hdr)[0]
    return msgpack.unpackb(_recvn(sock, n), raw=False)


def _recvn(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 22))
        if not chunk:
            raise ConnectionError("side channel closed")
        buf += chunk
    return bytes(buf)


@dataclass
class Held:
    seq_id: int
    blocks: list
    expiry: float
    num_tokens: int
    frees: set = field(default_factory=set)  # consumer TP ranks done reading
    swa_blocks: Optional[list] = None        # windowed pool of a hybrid cache


@dataclass
class LoadJob:
    request_id: str
    params: dict
    local_blocks: list
    t0: float = field(default_factory=time.monotonic)
    report: Optional[tuple] = None  # TP follower: the driver's side channel
    local_swa: Optional[list] = None  # hybrid cache: the windowed pool's destination blocks


def _pool_info(t: torch.Tensor) -> dict:
    """Geometry of a layer-major pool [L, num_blocks, planes, H, bs, D] in bytes."""
    esz = t.element_size()
    return {"shape": list(t.shape), "block_bytes": t[:, 0].numel() * esz,
            "layer_block_bytes": t[0, 0].numel() * esz, "layer_stride": t.stride(0) * esz}


LEGACY_IPC_MAX = 4 << 30  # hipIpcOpenMemHandle hangs importing larger allocations
RELAY_MB = int(os.environ.get("LLMD_KVX_RELAY_MB", "128"))  # staging per client decoder, two halves


def _hostport(x) -> tuple:
    if isinstance(x, (tuple, list)):
        return (str(x[0]), int(x[1]))
    h, p = str(x).rsplit(":", 1)
    return (h, int(p))


def stripe_plan(n: int, k: int) -> list[tuple[int, int]]:
    """Split n block pairs over 1 + k paths: [start, end) of the direct path first,
    then one range per relay (as equal as possible; empty ranges dropped)."""
    paths = 1 + k
    base, extra = divmod(n, paths)
    out, a = [], 0
    for i in range(paths):
        b = a + base + (1 if i < extra else 0)
        out.append((a, b))
        a = b
    return out

_P2P_GROUP = None  # torch.distributed group spanning prefill + decode engines (rccl transport)
# Held by the engine thread while it enqueues a forward pass (ModelRunner.run_plan) and by the
# kvx threads while they enqueue an rccl send / recv: the p2p communicator's operations are
# issued only between forward passes, never interleaved with a step's TP / EP collectives from
# another thread, so every rank issues its communicators' operations in one fixed order
# (two communicators driven from two threads in racing orders can deadlock).
_P2P_STEP_LOCK = threading.RLock()


class _NoGuard:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_NO_GUARD = _NoGuard()


def p2p_step_guard():
    """Context held around forward-pass enqueue; a no-op unless the rccl transport is set up."""
    return _P2P_STEP_LOCK if _P2P_GROUP is not None else _NO_GUARD


def set_p2p_group(group):
    """Register the process group the ``rccl`` transport sends over. Every rank of
    the world must create it (``dist.new_group``) before the engines start; it
    must not be used for anything else."""
    global _P2P_GROUP
    _P2P_GROUP = group


def p2p_group():
    return _P2P_GROUP


class _P2PSender:
    """Prefiller side of the rccl transport: ONE thread owns every send, in the
    order the pushes arrived (per decoder that is the order of its recvs)."""

    def __init__(self, agent: "KvxAgent"):
        self.agent = agent
        self.q: "queue.Queue[Optional[tuple]]" = queue.Queue()
        self.t = threading.Thread(target=self._run, daemon=True, name="kvx-p2p-send")
        self.t.start()

    def _run(self):
        import torch.distributed as dist

        a = self.agent
        stream = None
        while True:
            item = self.q.get()
            if item is None:
                return
            blocks, dst, pool = item
            try:
                if a.is_gpu:
                    if stream is None:
                        torch.cuda.set_device(a.kv.device)
                        stream = torch.cuda.Stream(device=a.kv.device)
                    with _P2P_STEP_LOCK, torch.cuda.stream(stream):  # enqueue between forward passes
                        buf = a.pack_blocks(blocks, pool)
                        dist.send(buf, dst=dst, group=_P2P_GROUP)
                    stream.synchronize()
                else:
                    with _P2P_STEP_LOCK:
                        dist.send(a.pack_blocks(blocks, pool), dst=dst, group=_P2P_GROUP)
            except Exception as e:  # noqa: BLE001 - the decoder's recv fails / times out in turn
                log.warning("kvx p2p send of %d blocks to rank %d failed: %s", len(blocks), dst, e)

    def close(self):
        self.q.put(None)


class KvxAgent:
    def __init__(self, kv: torch.Tensor, engine_id: Optional[str] = None, host: Optional[str] = None,
                 port: int = 0, tp_rank: int = 0, tp_size: int = 1, abort_timeout: float = 480.0,
                 transport: str = "auto", metrics=None, vmm: Optional[dict] = None, exports: bool = True,
                 workers: Optional[int] = None, require_ipc: bool = False, kv_swa: Optional[torch.Tensor] = None,
                 relays: Optional[list] = None, stripe_min_bytes: Optional[int] = None):
        self.kv = kv                      # [L, num_blocks, planes, Hkv, bs, D] (layer-major)
        self.kv_swa = kv_swa              # hybrid cache: the windowed layers' pool (same layout)
        self.require_ipc = require_ipc    # never degrade a GPU pull to TCP (bench / production P/D)
        env_relays = [x for x in os.environ.get("LLMD_KVX_RELAYS", "").split(",") if x]
        self.relays = [_hostport(r) for r in (relays if relays is not None else env_relays)]
        self.stripe_min = int(stripe_min_bytes if stripe_min_bytes is not None
                              else os.environ.get("LLMD_KVX_STRIPE_MIN_BYTES", str(64 << 20)))
        self.relay_bufs: dict[str, tuple] = {}  # relay role: per client engine, IPC-exported staging
        self.relay_lock = threading.Lock()
        self.relay_use: dict[tuple, threading.Lock] = {}  # decoder role: one pull at a time per relay
        self.vmm = vmm                    # chunked exportable pool (model_runner._alloc_cache)
        self.engine_id = engine_id or f"kvx-{uuid.uuid4().hex[:12]}"
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.abort_timeout = abort_timeout
        self.metrics = metrics
        self.is_gpu = kv.is_cuda
        esz = kv.element_size()
        self.block_bytes = kv[:, 0].numel() * esz        # one block, every layer
        self.layer_block_bytes = kv[0, 0].numel() * esz  # one block of one layer (pair stride)
        self.layer_stride = kv.stride(0) * esz           # one layer's pool
        self.transport = transport
        self.held: dict[str, Held] = {}
        self.held_lock = threading.Lock()
        self.free_requests: "queue.Queue[tuple]" = queue.Queue()
        self.done: "queue.Queue[tuple[str, bool]]" = queue.Queue()
        self.jobs: "queue.Queue[Optional[LoadJob]]" = queue.Queue()
        self.cancelled: set[str] = set()
        self.cancel_lock = threading.Lock()
        # TP driver: per request, [ranks reported, all ok] until every rank has
        self.tp_wait: dict[str, list] = {}
        self.tp_lock = threading.Lock()
        self.peers: dict[tuple, dict] = {}
        self.ipc_maps: dict[str, int] = {}
        self.ipc_handle = None
        self.ipc_handle_swa = None
        self.p2p_rank = None
        self.p2p_sender = None
        if _P2P_GROUP is not None:
            import torch.distributed as dist

            self.p2p_rank = dist.get_rank()
            if exports:
                self.p2p_sender = _P2PSender(self)
        self.p2p_lock = threading.Lock()  # decoder: one push + recv in flight per process
        self.uds_name = None
        if self.is_gpu and transport in ("auto", "ipc", "dma"):
            if vmm is not None:
                # hand the chunk fds to same-host peers over an abstract Unix socket
                self.uds_name = f"\0llmd-kvx-{self.engine_id}"
                self.uds = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                self.uds.bind(self.uds_name)
                self.uds.listen(16)
                threading.Thread(target=self._serve_fds, daemon=True, name="kvx-fds").start()
            elif kv.numel() * kv.element_size() <= LEGACY_IPC_MAX:
                try:
                    from llmd_amd.ops import native

                    h, off = native().kvx_ipc_export(kv)
                    self.ipc_handle = (h, off)
                except Exception as e:  # noqa: BLE001
                    log.warning("IPC export unavailable (%s); kvx falls back to TCP", e)
            elif exports:  # a pure consumer only pulls, nobody maps its pool
                log.warning("KV pool of %.1f GiB is not VMM-chunked; hipIpc cannot import >4 GiB, "
                            "kvx falls back to TCP", kv.numel() * kv.element_size() / 2**30)
            if kv_swa is not None and exports and kv_swa.numel() * kv_swa.element_size() <= LEGACY_IPC_MAX:
                try:
                    from llmd_amd.ops import native

                    h, off = native().kvx_ipc_export(kv_swa)
                    self.ipc_handle_swa = (h, off)
                except Exception as e:  # noqa: BLE001
                    log.warning("IPC export of the windowed pool unavailable (%s)", e)
        self.host = host or os.environ.get("VLLM_NIXL_SIDE_CHANNEL_HOST", "127.0.0.1")
        self.server = _Server(("0.0.0.0" if self.host not in ("127.0.0.1", "localhost") else self.host,
                               port or int(os.environ.get("VLLM_NIXL_SIDE_CHANNEL_PORT", "0") or 0)), self)
        self.port = self.server.server_address[1]
        threading.Thread(target=self.server.serve_forever, daemon=True, name="kvx-side-channel").start()
        self.peer_lock = threading.Lock()   # peers / ipc_maps setup, shared by the workers
        self._tls = threading.local()       # per-worker HIP stream
        self.n_workers = max(1, int(workers or os.environ.get("LLMD_KVX_WORKERS", "4")))
        self.workers = [threading.Thread(target=self._work, daemon=True, name=f"kvx-transfer-{i}")
                        for i in range(self.n_workers)]
        for t in self.workers:
            t.start()
        self.hb_interval = float(os.environ.get("LLMD_KVX_HEARTBEAT_S", "5"))
        self.hb_max_fails = int(os.environ.get("LLMD_KVX_HEARTBEAT_FAILS", "2"))
        self.hb_fails: dict[tuple, int] = {}
        self.known_peers: set[tuple] = set()
        self.dead_peers: set[tuple] = set()
        self._stop = threading.Event()
        if self.hb_interval > 0:
            threading.Thread(target=self._heartbeat, daemon=True, name="kvx-heartbeat").start()

    # ------------------------------------------------------------ liveness
    def ping(self, key: tuple, timeout: float = 2.0) -> bool:
        try:
            with socket.create_connection(key, timeout=timeout) as s:
                s.settimeout(timeout)
                _send(s, {"op": "ping"})
                return bool(_recv(s).get("ok"))
        except (OSError, ConnectionError, struct.error, ValueError):
            return False

    def heartbeat_once(self):
        for key in list(self.known_peers):
            if self.ping(key):
                self.hb_fails[key] = 0
                if key in self.dead_peers:
                    log.info("kvx peer %s:%d is back", *key)
                    self.dead_peers.discard(key)
                continue
            n = self.hb_fails.get(key, 0) + 1
            self.hb_fails[key] = n
            if n >= self.hb_max_fails and key not in self.dead_peers:
                log.warning("kvx peer %s:%d missed %d heartbeats: marking dead", key[0], key[1], n)
                self.dead_peers.add(key)
                p = self.peers.pop(key, None)
                if p is not None:
                    try:
                        p["sock"].close()
                    except OSError:
                        pass

    def _heartbeat(self):
        while not self._stop.wait(self.hb_interval):
            self.heartbeat_once()

    def peer_status(self) -> dict:
        return {f"{h}:{p}": ("dead" if (h, p) in self.dead_peers else "alive") for h, p in self.known_peers}

    def _serve_fds(self):
        fds = self.vmm["fds"]
        while True:
            try:
                c, _ = self.uds.accept()
            except OSError:
                return
            try:
                socket.send_fds(c, [struct.pack("<I", len(fds))], fds)
            except OSError:
                pass
            finally:
                c.close()

    # ------------------------------------------------------------ metadata
    def meta(self) -> dict:
        k = self.kv
        m = {"engine_id": self.engine_id, "shape": list(k.shape), "dtype": str(k.dtype).replace("torch.", ""),
             "block_bytes": self.block_bytes, "layout": "layer_major", "layer_block_bytes": self.layer_block_bytes,
             "layer_stride": self.layer_stride, "tp_rank": self.tp_rank, "tp_size": self.tp_size,
             "device": k.device.index if k.is_cuda else -1, "hostname": socket.gethostname(),
             "pid": os.getpid(), "num_blocks": k.shape[1]}
        if self.ipc_handle is not None:
            m["ipc_handle"], m["ipc_offset"] = self.ipc_handle
        if self.p2p_sender is not None:
            m["p2p_rank"] = self.p2p_rank
        if self.is_gpu and RELAY_MB > 0:
            m["relay"] = {"bytes": RELAY_MB << 20}
        if self.kv_swa is not None:
            m["swa"] = _pool_info(self.kv_swa)
            if self.ipc_handle_swa is not None:
                m["swa"]["ipc_handle"], m["swa"]["ipc_offset"] = self.ipc_handle_swa
        if self.uds_name is not None:
            off = self.kv.data_ptr() - self.vmm["pool"].data_ptr()
            m["vmm"] = {"uds": self.uds_name, "chunk": self.vmm["chunk"], "n": self.vmm["n"], "offset": off}
        return m

    # ------------------------------------------------------------ prefill side
    def hold(self, request_id: str, seq_id: int, blocks: list, num_tokens: int,
             swa_blocks: Optional[list] = None) -> dict:
        swa = list(swa_blocks) if swa_blocks is not None else None
        with self.held_lock:
            self.held[request_id] = Held(seq_id, list(blocks), time.monotonic() + self.abort_timeout, num_tokens,
                                         swa_blocks=swa)
        out = {"do_remote_prefill": True, "do_remote_decode": False, "remote_engine_id": self.engine_id,
               "remote_host": self.host, "remote_port": self.port, "remote_block_ids": list(blocks),
               "remote_request_id": request_id, "remote_tp_size": self.tp_size, "num_tokens": num_tokens}
        if swa is not None:
            out["remote_swa_block_ids"] = swa
        return out

    def expired_or_freed(self) -> list[Held]:
        """Held entries to release now (engine thread)."""
        out = []
        now = time.monotonic()
        while True:
            try:
                rid, rank, of = self.free_requests.get_nowait()
            except queue.Empty:
                break
            with self.held_lock:
                h = self.held.get(rid)
                if h is None:
                    continue
                h.frees.add(rank)
                if len(h.frees) < of:
                    continue  # other decoder TP ranks still read these blocks
                del self.held[rid]
            out.append(h)
        with self.held_lock:
            for rid in [r for r, h in self.held.items() if h.expiry < now]:
                log.warning("kvx: request %s held blocks expired (no remote read)", rid)
                out.append(self.held.pop(rid))
        return out

    def _pool(self, pool: str = "full") -> torch.Tensor:
        if pool == "swa":
            if self.kv_swa is None:
                raise RuntimeError("kvx: no windowed pool on this agent")
            return self.kv_swa
        return self.kv

    def pack_blocks(self, blocks: list, pool: str = "full") -> torch.Tensor:
        """Wire format: each block's bytes block-major [L, planes, H, bs, D], as one
        contiguous uint8 tensor on the pool's device."""
        kv = self._pool(pool)
        idx = torch.tensor(blocks, dtype=torch.long, device=kv.device)
        g = kv.index_select(1, idx).transpose(0, 1).contiguous()
        return g.view(torch.uint8).view(-1)

    def read_blocks(self, blocks: list, pool: str = "full") -> bytes:
        """Wire format (TCP path), as bytes."""
        return self.pack_blocks(blocks, pool).cpu().numpy().tobytes()

    # ------------------------------------------------------------ decode side
    def start_load(self, request_id: str, params: dict, local_blocks: list, report: Optional[tuple] = None,
                   local_swa: Optional[list] = None):
        """Queue a pull. ``report`` (TP followers) is the driver's side-channel
        address: completion goes there instead of this agent's ``done``.
        ``local_swa`` (or ``local_blocks.swa``): windowed-pool destinations."""
        if local_swa is None:
            local_swa = getattr(local_blocks, "swa", None)
        if self.tp_size > 1 and report is None:
            with self.tp_lock:
                self.tp_wait[request_id] = [0, True]
        self.jobs.put(LoadJob(request_id, dict(params), list(local_blocks), report=report,
                              local_swa=list(local_swa) if local_swa is not None else None))

    def _complete(self, job: LoadJob, ok: bool):
        if job.report is not None:
            try:
                with socket.create_connection(tuple(job.report), timeout=10) as s:
                    _send(s, {"op": "tp_done", "request_id": job.request_id, "ok": bool(ok)})
                    _recv(s)
            except (OSError, ConnectionError, struct.error) as e:
                log.warning("kvx: cannot report %s to the TP driver: %s", job.request_id, e)
            return
        self.tp_report(job.request_id, ok)

    def tp_report(self, request_id: str, ok: bool):
        """One TP rank (this one, or a follower over ``tp_done``) finished."""
        if self.tp_size == 1:
            self.done.put((request_id, ok))
            return
        with self.tp_lock:
            w = self.tp_wait.setdefault(request_id, [0, True])
            w[0] += 1
            w[1] = w[1] and ok
            if w[0] < self.tp_size:
                return
            del self.tp_wait[request_id]
        self.done.put((request_id, w[1]))

    def cancel(self, request_id: str):
        with self.cancel_lock:
            self.cancelled.add(request_id)

    def _take_cancel(self, request_id: str) -> bool:
        with self.cancel_lock:
            if request_id in self.cancelled:
                self.cancelled.discard(request_id)
                return True
            return False

    def _notify_free(self, prm: dict):
        """Abort notif: tell the prefiller it can release the held blocks."""
        try:
            p = self._peer(prm["remote_host"], prm["remote_port"])
            self._rpc(p, self._free_msg(prm))
        except Exception as e:  # noqa: BLE001 - the prefiller's abort timeout reclaims them
            log.warning("kvx abort notif for %s failed: %s", prm.get("remote_request_id"), e)

    def _free_msg(self, prm: dict) -> dict:
        return {"op": "free", "request_id": prm.get("remote_request_id"), "rank": self.tp_rank,
                "of": self.tp_size}

    def _peer(self, host, port) -> dict:
        key = (host, int(port))
        self.known_peers.add(key)
        if key in self.dead_peers:
            raise RuntimeError(f"prefiller {host}:{port} failed its heartbeat")
        with self.peer_lock:
            p = self.peers.get(key)
            if p is None:
                s = socket.create_connection(key, timeout=10)
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                _send(s, {"op": "meta"})
                meta = _recv(s)
                p = {"sock": s, "meta": meta, "lock": threading.Lock()}
                self._check_compat(meta)
                self.peers[key] = p
        return p

    def _check_compat(self, m: dict):
        """Handshake compatibility (enforce_handshake_compat): layout, block size,
        dtype, layers, head dim must match; KV heads may differ by TP re-slicing."""
        ls = list(self.kv.shape)
        rs = m["shape"]
        if m.get("layout") != "layer_major":
            raise RuntimeError("kvx: peer KV pool is not layer-major (incompatible version)")
        if rs[0] != ls[0] or rs[2] != ls[2] or rs[4] != ls[4] or rs[5] != ls[5]:
            raise RuntimeError(f"kvx layout mismatch local {ls} remote {rs}")
        if m["dtype"] != str(self.kv.dtype).replace("torch.", ""):
            raise RuntimeError("kvx dtype mismatch")
        if ("swa" in m) != (self.kv_swa is not None):
            raise RuntimeError("kvx: hybrid (windowed-pool) KV cache on one side only; run both engines with "
                               "the same --disable-hybrid-kv-cache-manager setting")
        if "swa" in m:
            rw, lw = m["swa"]["shape"], list(self.kv_swa.shape)
            if rw[0] != lw[0] or rw[2] != lw[2] or rw[4] != lw[4] or rw[5] != lw[5]:
                raise RuntimeError(f"kvx windowed-pool layout mismatch local {lw} remote {rw}")
        if rs[3] % ls[3] and ls[3] % rs[3]:
            raise RuntimeError("kvx: KV head counts not TP-compatible")

    def _rpc(self, p, obj):
        with p["lock"]:
            _send(p["sock"], obj)
            return _recv(p["sock"])

    def _head_slice(self, rmeta) -> tuple[int, int, int]:
        """(remote heads, local heads, first remote head of this rank's slice)."""
        hl, hr = self.kv.shape[3], rmeta["shape"][3]
        if hr < hl:
            raise RuntimeError("kvx: decoder holds more KV heads than the prefiller (unsupported pull)")
        return hr, hl, (self.tp_rank * hl) % hr  # prefiller has all heads of a group of decoder ranks

    @staticmethod
    def _rinfo(rmeta, pool: str = "full") -> dict:
        return rmeta["swa"] if pool == "swa" else rmeta

    def _segments(self, rmeta, pool: str = "full") -> list[tuple[int, int, int]]:
        """IPC copy segments (src_off, dst_off, len) of one block, relative to
        block * layer_block_bytes in each pool: one per layer (per layer and
        plane when TP re-slices heads) - a block is 2 L pieces of the
        layer-major pools."""
        kv = self._pool(pool)
        ri = self._rinfo(rmeta, pool)
        L, _, planes, _, bs, D = kv.shape
        hr, hl, h0 = self._head_slice(rmeta)
        esz = kv.element_size()
        lsr, lsl = int(ri["layer_stride"]), kv.stride(0) * esz
        lbb = kv[0, 0].numel() * esz
        if hr == hl:
            return [(l * lsr, l * lsl, lbb) for l in range(L)]
        head = bs * D * esz
        return [(l * lsr + (p * hr + h0) * head, l * lsl + p * hl * head, hl * head)
                for l in range(L) for p in range(planes)]

    def _wire_segments(self, rmeta, pool: str = "full") -> list[tuple[int, int, int]]:
        """TCP / rccl paths: segments inside one block-major wire block (read_blocks)."""
        kv = self._pool(pool)
        L, _, planes, _, bs, D = kv.shape
        hr, hl, h0 = self._head_slice(rmeta)
        if hr == hl:
            return [(0, 0, kv[:, 0].numel() * kv.element_size())]
        head = bs * D * kv.element_size()
        return [(((l * planes + p) * hr + h0) * head, ((l * planes + p) * hl) * head, hl * head)
                for l in range(L) for p in range(planes)]

    def _fault(self) -> Optional[str]:
        f = os.environ.get("LLMD_KVX_FAULT")
        if not f or random.random() > float(os.environ.get("LLMD_KVX_FAULT_P", "1.0")):
            return None
        return f

    def _work(self):
        while True:
            job = self.jobs.get()
            if job is None:
                return
            ok = False
            t0 = time.monotonic()
            nbytes = 0
            if self._take_cancel(job.request_id):
                # aborted before the pull started: nothing was written locally
                self._notify_free(job.params)
                self._complete(job, False)
                continue
            mk = markers.start(f"llmd.kvx.pull {job.request_id}")
            try:
                ok, nbytes = self._do_load(job)
            except Exception as e:  # noqa: BLE001 - NIXL_ERR_BACKEND equivalent
                log.warning("kvx load %s failed: %s", job.request_id, e)
                ok = False
            markers.stop(mk)
            if self.metrics is not None:
                self.metrics.observe(ok, time.monotonic() - t0, nbytes, len(job.local_blocks))
            self._take_cancel(job.request_id)  # a cancel that raced the running pull
            self._complete(job, ok)

    def _do_load(self, job: LoadJob) -> tuple[bool, int]:
        prm = job.params
        fault = self._fault()
        if fault == "drop":
            raise RuntimeError("injected transfer drop")
        if fault and fault.startswith("delay:"):
            time.sleep(float(fault.split(":")[1]))
        p = self._peer(prm["remote_host"], prm["remote_port"])
        rmeta = p["meta"]
        rblocks = list(prm["remote_block_ids"])
        n = min(len(rblocks), len(job.local_blocks))
        # (pool, remote blocks, local blocks): the windowed pool of a hybrid cache moves
        # only the pairs both sides hold (null = block 0 before the last window)
        work = [("full", rblocks[:n], job.local_blocks[:n])]
        rs, ls = prm.get("remote_swa_block_ids"), job.local_swa
        if self.kv_swa is not None and rs is not None and ls is not None:
            pairs = [(r, l) for r, l in zip(rs, ls) if r and l]
            if pairs:
                work.append(("swa", [r for r, _ in pairs], [l for _, l in pairs]))
        elif (self.kv_swa is not None) != (rs is not None):
            raise RuntimeError("kvx: request and KV cache disagree on the hybrid (windowed) pool")
        use_ipc = (self.is_gpu and ("ipc_handle" in rmeta or "vmm" in rmeta)
                   and self.transport in ("auto", "ipc", "dma") and not p.get("no_ipc")
                   and rmeta.get("hostname") == socket.gethostname()
                   and (len(work) == 1 or "ipc_handle" in rmeta.get("swa", {})))
        nbytes = sum(sum(sg[2] for sg in self._segments(rmeta, pool)) * len(lb) for pool, _, lb in work)
        use_p2p = (self.transport == "rccl" and _P2P_GROUP is not None and rmeta.get("p2p_rank") is not None)
        if self.transport == "rccl" and not use_p2p:
            raise RuntimeError(f"kvx: rccl transport to {rmeta.get('engine_id')} needs a shared p2p group "
                               f"(set_p2p_group) and a sending peer (peer p2p rank {rmeta.get('p2p_rank')})")
        if use_p2p:
            for pool, rb, lb in work:
                self._p2p_pull(p, prm, rb, lb, pool)
            use_ipc = False
        elif self.require_ipc and self.is_gpu and not use_ipc and self.transport != "tcp":
            raise RuntimeError(f"kvx: no IPC path to {rmeta.get('engine_id')} (host {rmeta.get('hostname')}, "
                               f"handle {'ipc_handle' in rmeta or 'vmm' in rmeta}, degraded {bool(p.get('no_ipc'))}) "
                               "and require_ipc is set")
        if use_ipc:
            try:
                for pool, rb, lb in work:
                    sg = self._segments(rmeta, pool)
                    if pool == "full" and self._striped_ipc_copy(rmeta, rb, lb, sg):
                        continue
                    self._ipc_copy(rmeta, rb, lb, sg, pool)
            except Exception as e:  # noqa: BLE001 - mapping failed: degrade this peer to TCP
                if self.require_ipc:
                    raise RuntimeError(f"kvx IPC pull from {rmeta.get('engine_id')} failed: {e}") from e
                log.warning("kvx IPC path to %s failed (%s); using TCP for this peer", rmeta.get("engine_id"), e)
                p["no_ipc"] = True
                use_ipc = False
                if self.metrics is not None and hasattr(self.metrics, "on_ipc_fallback"):
                    self.metrics.on_ipc_fallback()
        if not use_ipc and not use_p2p:
            for pool, rb, lb in work:
                data = self._rpc(p, {"op": "read", "blocks": rb, "request_id": prm.get("remote_request_id"),
                                     "pool": pool})
                if isinstance(data, dict) and data.get("error"):
                    raise RuntimeError(data["error"])
                src = torch.frombuffer(bytearray(data), dtype=torch.uint8).view(len(rb), -1)
                self._scatter_wire(rmeta, src, lb, pool)
            if self.is_gpu:
                torch.cuda.current_stream().synchronize()
        if fault == "corrupt":
            idx = torch.tensor(work[0][2][:1], dtype=torch.long, device=self.kv.device)
            self.kv.index_fill_(1, idx, 0)
        # release the prefiller's blocks (this rank's share)
        self._rpc(p, self._free_msg(prm))
        return True, nbytes

    def _scatter_wire(self, rmeta, src: torch.Tensor, lblocks: list, pool: str = "full"):
        """Write wire-format blocks ``src`` [n, remote block bytes] (any device) into the
        local pool at ``lblocks`` (this rank's head slice)."""
        kv = self._pool(pool)
        n = len(lblocks)
        dst_idx = torch.tensor(lblocks, dtype=torch.long, device=kv.device)
        segs = self._wire_segments(rmeta, pool)
        bb = kv[:, 0].numel() * kv.element_size()
        if len(segs) == 1 and segs[0][2] == src.shape[1]:
            rows = src
        else:
            rows = torch.empty(n, bb, dtype=torch.uint8, device=src.device)
            for so, do, ln in segs:
                rows[:, do:do + ln] = src[:, so:so + ln]
        blk = rows.view(kv.dtype).view((n,) + tuple(kv.shape[:1]) + tuple(kv.shape[2:]))
        kv.index_copy_(1, dst_idx, blk.transpose(0, 1).to(kv.device))

    def _p2p_pull(self, p, prm, rblocks, lblocks, pool: str = "full"):
        """rccl transport: push request, then the matching recv, then the scatter."""
        import torch.distributed as dist

        rmeta = p["meta"]
        rbb = int(self._rinfo(rmeta, pool)["block_bytes"])
        n = len(rblocks)
        stream = None
        if self.is_gpu:
            stream = getattr(self._tls, "stream", None)
            if stream is None:
                torch.cuda.set_device(self.kv.device)
                stream = self._tls.stream = torch.cuda.Stream(device=self.kv.device)
        with self.p2p_lock:
            r = self._rpc(p, {"op": "push", "blocks": rblocks, "request_id": prm.get("remote_request_id"),
                              "dst": self.p2p_rank, "pool": pool})
            if not (isinstance(r, dict) and r.get("ok")):
                raise RuntimeError(f"kvx push refused: {r}")
            if stream is not None:
                with _P2P_STEP_LOCK, torch.cuda.stream(stream):  # enqueue between forward passes
                    buf = torch.empty(n * rbb, dtype=torch.uint8, device=self.kv.device)
                    dist.recv(buf, src=int(rmeta["p2p_rank"]), group=_P2P_GROUP)
                    self._scatter_wire(rmeta, buf.view(n, rbb), lblocks, pool)
                stream.synchronize()
            else:
                buf = torch.empty(n * rbb, dtype=torch.uint8)
                with _P2P_STEP_LOCK:
                    dist.recv(buf, src=int(rmeta["p2p_rank"]), group=_P2P_GROUP)
                self._scatter_wire(rmeta, buf.view(n, rbb), lblocks, pool)

    # ------------------------------------------------------------ relay (multi-link striping)
    def _relay_staging(self, client: str) -> tuple:
        """(staging tensor, (ipc handle, offset)) of one client decoder, created on first
        use (clients never share a staging buffer, so their chunks cannot collide)."""
        with self.relay_lock:
            st = self.relay_bufs.get(client)
            if st is None:
                from llmd_amd.ops import native

                buf = torch.empty(RELAY_MB << 20, dtype=torch.uint8, device=self.kv.device)
                h, off = native().kvx_ipc_export(buf)
                st = self.relay_bufs[client] = (buf, (bytes(h), int(off)))
            return st

    def relay_copy(self, src_meta: dict, pairs: list, segs: list, slot_bytes: int, half: int,
                   client: str = "") -> dict:
        """Relay side: copy blocks of a peer's pool (mapped here) into the client's
        staging half ``half``, packed at ``slot_bytes`` per block (one kernel, src ->
        this GPU)."""
        from llmd_amd.ops import native

        C = native()
        buf, (h, off) = self._relay_staging(client)
        halfb = buf.numel() // 2
        if len(pairs) * slot_bytes > halfb:
            raise RuntimeError(f"relay chunk of {len(pairs)} x {slot_bytes} B exceeds the staging half ({halfb} B)")
        stream = getattr(self._tls, "rstream", None)
        if stream is None:
            torch.cuda.set_device(self.kv.device)
            stream = self._tls.rstream = torch.cuda.Stream(device=self.kv.device)
        with self.peer_lock:
            base = self._map_peer(C, src_meta["engine_id"], src_meta)
        dst = buf[half * halfb:(half + 1) * halfb]
        with torch.cuda.stream(stream):
            pr = torch.tensor(pairs, dtype=torch.int32, device=self.kv.device)
            sg = torch.tensor(segs, dtype=torch.int64, device=self.kv.device)
            C.kvx_copy_blocks(dst, base, slot_bytes, int(src_meta["layer_block_bytes"]), pr, sg,
                              max(x[2] for x in segs), COPY_ENGINE)
        stream.synchronize()
        return {"ok": True, "ipc_handle": h, "ipc_offset": off, "half_bytes": halfb}

    def _relay_pull(self, relay: tuple, rmeta: dict, rblocks: list, lblocks: list, segs: list):
        """Decoder side of one relay path: chunks alternate between the relay's two
        staging halves; the relay's copy of chunk i+1 (P -> R) overlaps ours of chunk i
        (R -> D)."""
        from llmd_amd.ops import native

        C = native()
        rp = self._peer(*relay)
        # packed layout inside the staging: each block's segments back to back
        slot = sum(x[2] for x in segs)
        leg1, leg2, o = [], [], 0
        for so, do, ln in segs:
            leg1.append((so, o, ln))
            leg2.append((o, do, ln))
            o += ln
        half_bytes = (int(rp["meta"].get("relay", {}).get("bytes", RELAY_MB << 20)) // 2)
        per = max(1, half_bytes // slot)
        stream = getattr(self._tls, "stream", None)
        if stream is None:
            torch.cuda.set_device(self.kv.device)
            stream = self._tls.stream = torch.cuda.Stream(device=self.kv.device)
        src_meta = {k: v for k, v in rmeta.items() if k != "swa"}
        pending = [None, None]  # per half: event of our last copy out of it
        base = None
        with self.peer_lock:
            use = self.relay_use.setdefault(relay, threading.Lock())
        with use:  # one pull at a time through our staging on this relay
            self._relay_chunks(C, rp, relay, src_meta, rblocks, lblocks, leg1, leg2, slot, per, stream, pending)

    def _relay_chunks(self, C, rp, relay, src_meta, rblocks, lblocks, leg1, leg2, slot, per, stream, pending):
        base = None
        for ci, a in enumerate(range(0, len(rblocks), per)):
            b = min(len(rblocks), a + per)
            half = ci & 1
            if pending[half] is not None:
                pending[half].synchronize()  # the relay may overwrite this half only once we read it
            r = self._rpc(rp, {"op": "relay_copy", "src": src_meta, "segs": leg1, "slot_bytes": slot, "half": half,
                               "pairs": [[rb, i] for i, rb in enumerate(rblocks[a:b])], "client": self.engine_id})
            if not (isinstance(r, dict) and r.get("ok")):
                raise RuntimeError(f"kvx relay {relay[0]}:{relay[1]} failed: {r}")
            if base is None:
                key = f"relay:{r['ipc_handle'].hex()}"
                with self.peer_lock:
                    base = self.ipc_maps.get(key)
                    if base is None:
                        base = self.ipc_maps[key] = C.kvx_ipc_open(r["ipc_handle"]) + int(r["ipc_offset"])
            with torch.cuda.stream(stream):
                pr = torch.tensor([[i, lb] for i, lb in enumerate(lblocks[a:b])], dtype=torch.int32,
                                  device=self.kv.device)
                sg = torch.tensor(leg2, dtype=torch.int64, device=self.kv.device)
                C.kvx_copy_blocks(self.kv, base + half * int(r["half_bytes"]), self.layer_block_bytes, slot, pr, sg,
                                  max(x[2] for x in leg2), COPY_ENGINE)
                ev = torch.cuda.Event()
                ev.record(stream)
            pending[half] = ev
        for ev in pending:
            if ev is not None:
                ev.synchronize()

    def _striped_ipc_copy(self, rmeta, rblocks, lblocks, segs) -> bool:
        """Full-pool pull over the direct link + every relay, concurrently. False if
        striping does not apply (no relays, small pull)."""
        nbytes = sum(x[2] for x in segs) * len(rblocks)
        if not self.relays or nbytes < self.stripe_min or len(rblocks) < 2:
            return False
        plan = stripe_plan(len(rblocks), len(self.relays))
        errs = []

        def leg(i, a, b):
            try:
                if i == 0:
                    self._ipc_copy(rmeta, rblocks[a:b], lblocks[a:b], segs)
                else:
                    self._relay_pull(self.relays[i - 1], rmeta, rblocks[a:b], lblocks[a:b], segs)
            except Exception as e:  # noqa: BLE001 - reported below
                errs.append(e)

        ts = [threading.Thread(target=leg, args=(i, a, b), daemon=True) for i, (a, b) in enumerate(plan) if b > a]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise RuntimeError(f"striped pull failed: {errs[0]}")
        if self.metrics is not None and hasattr(self.metrics, "on_striped"):
            self.metrics.on_striped(len(ts))
        return True

    def _ipc_copy(self, rmeta, rblocks, lblocks, segs, pool: str = "full"):
        from llmd_amd.ops import native

        C = native()
        eid = rmeta["engine_id"]
        kv = self._pool(pool)
        ri = self._rinfo(rmeta, pool)
        stream = getattr(self._tls, "stream", None)
        if stream is None:
            torch.cuda.set_device(self.kv.device)
            stream = self._tls.stream = torch.cuda.Stream(device=self.kv.device)
        with self.peer_lock:
            base = self._map_peer(C, eid, rmeta, pool)
        with torch.cuda.stream(stream):
            # block b of layer l sits at pool + l * layer_stride + b * layer_block_bytes
            pairs = torch.tensor(list(zip(rblocks, lblocks)), dtype=torch.int32, device=kv.device)
            sg = torch.tensor(segs, dtype=torch.int64, device=kv.device)
            C.kvx_copy_blocks(kv, base, kv[0, 0].numel() * kv.element_size(), int(ri["layer_block_bytes"]), pairs,
                              sg, max(x[2] for x in segs), COPY_ENGINE)
            ev = torch.cuda.Event()
            ev.record(stream)
        ev.synchronize()

    def _map_peer(self, C, eid, rmeta, pool: str = "full") -> int:
        """Base pointer of a peer's KV pool in this process (mapped once)."""
        if pool == "swa":
            key = eid + ":swa"
            base = self.ipc_maps.get(key)
            if base is None:
                sw = rmeta["swa"]
                base = self.ipc_maps[key] = C.kvx_ipc_open(sw["ipc_handle"]) + int(sw["ipc_offset"])
            return base
        base = self.ipc_maps.get(eid)
        if base is None:
            if "vmm" in rmeta:
                vm = rmeta["vmm"]
                c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                c.settimeout(30)
                c.connect(vm["uds"])
                _, fds, _, _ = socket.recv_fds(c, 16, int(vm["n"]))
                c.close()
                try:
                    base = C.vmm_import(list(fds), int(vm["chunk"]), self.kv.device.index) + int(vm["offset"])
                finally:
                    for fd in fds:
                        os.close(fd)
            else:
                base = C.kvx_ipc_open(rmeta["ipc_handle"]) + int(rmeta["ipc_offset"])
            self.ipc_maps[eid] = base
        return base

    def poll_done(self) -> list[tuple[str, bool]]:
        out = []
        while True:
            try:
                out.append(self.done.get_nowait())
            except queue.Empty:
                return out

    def close(self):
        self._stop.set()
        if self.p2p_sender is not None:
            self.p2p_sender.close()
        for _ in self.workers:
            self.jobs.put(None)
        self.server.shutdown()
        for p in self.peers.values():
            try:
                p["sock"].close()
            except OSError:
                pass
        # peer pools mapped into this process (self.ipc_maps) stay mapped until
        # process exit: a pull kernel may still reference them on another stream


def _held_ok(agent: KvxAgent, msg: dict, pool: str) -> bool:
    """A read / push may only name blocks the request holds (of that pool)."""
    with agent.held_lock:
        held = agent.held.get(msg.get("request_id"))
    if held is None:
        return True
    have = held.swa_blocks if pool == "swa" else held.blocks
    return have is not None and set(msg["blocks"]) <= set(have)


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        agent: KvxAgent = self.server.agent
        s = self.request
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        while True:
            try:
                msg = _recv(s)
            except (ConnectionError, OSError, struct.error):
                return
            op = msg.get("op")
            try:
                if op == "meta":
                    _send(s, agent.meta())
                elif op == "read":
                    pool = msg.get("pool", "full")
                    if not _held_ok(agent, msg, pool):
                        _send(s, {"error": "blocks not held for request"})
                        continue
                    _send(s, agent.read_blocks(msg["blocks"], pool))
                elif op == "push":  # rccl transport: queue the send, the decoder posts the recv
                    pool = msg.get("pool", "full")
                    if agent.p2p_sender is None:
                        _send(s, {"error": "no p2p group on this agent"})
                    elif not _held_ok(agent, msg, pool):
                        _send(s, {"error": "blocks not held for request"})
                    else:
                        agent.p2p_sender.q.put((list(msg["blocks"]), int(msg["dst"]), pool))
                        _send(s, {"ok": True})
                elif op == "free":
                    agent.free_requests.put((msg.get("request_id"), int(msg.get("rank", 0)),
                                             int(msg.get("of", 1))))
                    _send(s, {"ok": True})
                elif op == "relay_copy":  # multi-link striping: this agent relays a share of a pull
                    try:
                        _send(s, agent.relay_copy(msg["src"], msg["pairs"], msg["segs"], int(msg["slot_bytes"]),
                                                  int(msg["half"]), str(msg.get("client", ""))))
                    except Exception as e:  # noqa: BLE001 - the decoder fails the pull (-> failure policy)
                        _send(s, {"error": f"relay: {e}"})
                elif op == "tp_done":
                    agent.tp_report(msg["request_id"], bool(msg.get("ok")))
                    _send(s, {"ok": True})
                elif op == "ping":
                    _send(s, {"ok": True, "engine_id": agent.engine_id})
                else:
                    _send(s, {"error": f"unknown op {op}"})
            except (ConnectionError, OSError):
                return


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, addr, agent):
        self.agent = agent
        super().__init__(addr, _Handler)
