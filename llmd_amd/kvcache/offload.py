"""Tiered KV offload: GPU -> pinned host DRAM -> filesystem (SURVEY N14-N16,
C-M15; docs/architecture/advanced/kv-management/kv-offloader.md).

Policy: *write-through*. A block is immutable once full, so as soon as the
engine commits a full block (BlockStored) it is copied D2H on a dedicated
low-priority HIP stream (ordered after the compute stream that produced it)
into a pinned host pool; no copy is ever on the eviction critical path.
The host tier is an LRU over block keys (``cpu_bytes_to_use``); with an FS
tier configured, host-resident blocks are also persisted as one file per block
(``<root>/<key[:2]>/<key>.kv``) by the native C++ write pool straight from the
pinned slot (zero-copy: the slot is pinned against eviction until the write
lands), so KV survives engine restarts (the llm-d FS connector behaviour).

Reloads are asynchronous, like the reference offloader's DMA workers
(kv-offloader.md:21,104-136): on admission the scheduler calls
``start_load``; blocks continuing the request's GPU-cached prefix are looked up
host-then-disk, destination blocks are allocated, FS blocks are read by the
native read pool into pinned buffers, then everything is copied H2D and
scattered into the pool on the side stream. The request waits in the
scheduler's ``offload_wait`` while the engine keeps stepping other requests;
``poll_loads`` hands it back (with the loaded tokens counted as computed) once
the side stream's event has fired. Nothing on the engine thread blocks on disk
or on the copy engines.

The device pool is layer-major ([L, num_blocks, 2, Hkv, bs, D], see
engine/model_runner.py); a host slot holds one block block-major
([L, 2, Hkv, bs, D], ``block_bytes``). The gather into (and scatter out of) a
contiguous staging slab is one launch of the LDS-staged block-copy kernel
(csrc/ops/kvx_copy.hip, the K17 "contiguous all-layer layout for one DMA").

Tier changes are published as KV events with ``medium`` cpu / disk so the
router's precise index scores them with tier weights. Transfer metrics use
vLLM's ``vllm:kv_offload_*`` names (bytes, time, size distribution per
transfer type; kv-offloader.md:211).
"""
from __future__ import annotations

import collections
import hashlib
import itertools
import logging
import threading
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from llmd_amd import _rt_loader

log = logging.getLogger("llmd.offload")

# transfer-size histogram buckets (bytes): one observation per batched transfer
_SIZE_BUCKETS = [1 << 16, 1 << 18, 1 << 20, 1 << 22, 1 << 24, 1 << 26, 1 << 28, 1 << 30, 1 << 32]
_XFER_TYPES = ("GPU_to_CPU", "CPU_to_GPU", "CPU_to_FS", "FS_to_CPU")


class _XferStats:
    """vllm:kv_offload_total_bytes / _total_time (counters) and vllm:kv_offload_size
    (histogram) per transfer type."""

    def __init__(self):
        self.bytes = {t: 0 for t in _XFER_TYPES}
        self.secs = {t: 0.0 for t in _XFER_TYPES}
        self.hist = {t: [0] * (len(_SIZE_BUCKETS) + 1) for t in _XFER_TYPES}
        self.hsum = {t: 0 for t in _XFER_TYPES}

    def add(self, kind: str, nbytes: int, secs: float, observe: bool = True):
        self.bytes[kind] += int(nbytes)
        self.secs[kind] += float(secs)
        if observe and nbytes:
            i = next((k for k, b in enumerate(_SIZE_BUCKETS) if nbytes <= b), len(_SIZE_BUCKETS))
            self.hist[kind][i] += 1
            self.hsum[kind] += int(nbytes)

    def render(self, lab: str) -> list[str]:
        out = ["# HELP vllm:kv_offload_total_bytes Bytes moved by the KV offload tiers",
               "# TYPE vllm:kv_offload_total_bytes counter"]
        out += [f'vllm:kv_offload_total_bytes{{{lab},transfer_type="{t}"}} {self.bytes[t]}' for t in _XFER_TYPES]
        out += ["# HELP vllm:kv_offload_total_time Seconds spent in KV offload transfers",
                "# TYPE vllm:kv_offload_total_time counter"]
        out += [f'vllm:kv_offload_total_time{{{lab},transfer_type="{t}"}} {self.secs[t]:.6f}' for t in _XFER_TYPES]
        out += ["# HELP vllm:kv_offload_size Size of KV offload transfers (bytes)",
                "# TYPE vllm:kv_offload_size histogram"]
        for t in _XFER_TYPES:
            acc = 0
            for b, c in zip(_SIZE_BUCKETS + [None], self.hist[t]):
                acc += c
                le = "+Inf" if b is None else f"{float(b):.1f}"
                out.append(f'vllm:kv_offload_size_bucket{{{lab},transfer_type="{t}",le="{le}"}} {acc}')
            out.append(f'vllm:kv_offload_size_count{{{lab},transfer_type="{t}"}} {acc}')
            out.append(f'vllm:kv_offload_size_sum{{{lab},transfer_type="{t}"}} {self.hsum[t]}')
        return out


@dataclass
class _LoadJob:
    req: object
    first: int                      # first block index (in the request's table) being loaded
    dst: list                       # destination pool block ids
    items: list                     # (tier, key, slot | pinned buffer)
    fs_tickets: set = field(default_factory=set)
    n_ok: int = -1                  # blocks usable (a failed FS read truncates the prefix)
    event: object = None            # side-stream completion event (GPU)
    keep: tuple = ()                # staging tensors referenced until the event fires
    t0: float = 0.0
    ev0: object = None
    aborted: bool = False
    released: bool = False          # host-slot references given back (poll_loads / cancel)


def _slot_runs(slots: list):
    """(first index, first slot, length) of each run of consecutive host slots, so a
    multi-block transfer is one copy per run instead of one per block."""
    out = []
    i = 0
    while i < len(slots):
        r = 1
        while i + r < len(slots) and slots[i + r] == slots[i] + r:
            r += 1
        out.append((i, slots[i], r))
        i += r
    return out


class OffloadManager:
    def __init__(self, cfg, engine, pool: str = "full", cpu_share: float = 1.0):
        oc = dict(cfg.kv_offload_config or {})
        extra = oc.get("kv_connector_extra_config", oc)
        self.engine = engine
        self.pool = pool  # "full": the main pool; "swa": the windowed pool of a hybrid cache
        self.kv = engine.runner.kv if pool == "full" else engine.runner.kv_swa
        self._layout(self.kv)
        cpu_bytes = int(int(extra.get("cpu_bytes_to_use", extra.get("cpu_bytes", 1 << 30))) * cpu_share)
        self.n_slots = max(1, cpu_bytes // self.block_bytes)
        pin = self.kv.is_cuda
        self.host = torch.empty(self.n_slots, self.block_bytes, dtype=torch.uint8, pin_memory=pin)
        self.slot_of: "collections.OrderedDict[int, int]" = collections.OrderedDict()  # key -> slot (LRU)
        self.free_slots = list(range(self.n_slots - 1, -1, -1))
        # slots that must not be recycled: FS write from the slot in flight, or a reload reading it
        self.slot_busy: collections.Counter = collections.Counter()
        self.pending: list = []  # write-through copies in flight
        self.fs = None
        fs = extra.get("fs_root") or next((t.get("root_dir") for t in extra.get("secondary_tiers", [])
                                           if t.get("type") == "fs"), None)
        if fs:
            rt = _rt_loader.rt()
            tiers = {t.get("type"): t for t in extra.get("secondary_tiers", [])}
            ft = tiers.get("fs", {})
            wthreads = int(extra.get("n_write_threads", ft.get("n_write_threads", 8)))
            rthreads = int(extra.get("n_read_threads", ft.get("n_read_threads", 8)))
            self.fs = rt.FsStore(fs, wthreads, rthreads)
        self._fs_io0 = [0.0, 0.0, 0.0, 0.0]
        self.fs_writes: dict[int, int] = {}     # ticket -> slot
        self._ticket = itertools.count(1)
        self.loads: dict[str, _LoadJob] = {}  # request id -> job
        self._fs_read_job: dict[int, _LoadJob] = {}
        self.stream = torch.cuda.Stream(priority=0) if self.kv.is_cuda else None
        self.events_out: list = []
        self.stats = {"offloaded": 0, "loaded_cpu": 0, "loaded_fs": 0, "evicted_cpu": 0}
        self.xfer = _XferStats()
        self.lock = threading.Lock()
        # FS keys carry a namespace derived from the weights' stable identity
        # (engine/weight_sync.py: checkpoint identity, trainer version or a unique
        # id per update), not a per-process counter: a restarted engine, or another
        # replica sharing fs_root, only ever reads KV computed by the same weights
        self.weights_id = engine.weight_sync.weights_id
        self.ns = self._namespace(self.weights_id)

    def _layout(self, kv):
        """Block geometry of the layer-major pool and the copy segments that move one
        block between it and a block-major slab row (pack / unpack)."""
        L, NB = kv.shape[0], kv.shape[1]
        self.block_bytes = kv[:, 0].numel() * kv.element_size()
        self.blk_shape = (L,) + tuple(kv.shape[2:])  # one block, block-major
        self.layer_block_bytes = self.block_bytes // L
        lbb, lstride = self.layer_block_bytes, NB * self.layer_block_bytes
        self._pack_segs = [(l * lstride, l * lbb, lbb) for l in range(L)]
        self._unpack_segs = [(l * lbb, l * lstride, lbb) for l in range(L)]
        self._segs_dev = None

    @staticmethod
    def _namespace(weights_id: str) -> str:
        return hashlib.sha256(weights_id.encode()).hexdigest()[:12]

    def _fs_key(self, h: int) -> str:
        return f"{h:016x}-{self.ns}" + ("-swa" if self.pool == "swa" else "")

    # ------------------------------------------------------------ slab pack / unpack
    def _seg_tensors(self):
        if self._segs_dev is None:
            dev = self.kv.device
            self._segs_dev = (torch.tensor(self._pack_segs, dtype=torch.int64, device=dev),
                              torch.tensor(self._unpack_segs, dtype=torch.int64, device=dev))
        return self._segs_dev

    def _pack(self, blocks: list) -> torch.Tensor:
        """[n, block_bytes] uint8 staging slab of the given pool blocks (current stream)."""
        n = len(blocks)
        if not self.kv.is_cuda:
            idx = torch.tensor(blocks, dtype=torch.long)
            return self.kv.index_select(1, idx).transpose(0, 1).contiguous().view(n, -1).view(torch.uint8)
        from llmd_amd.kvx.agent import COPY_ENGINE
        from llmd_amd.ops import native

        stage = torch.empty(n, self.block_bytes, dtype=torch.uint8, device=self.kv.device)
        pairs = torch.tensor([[b, j] for j, b in enumerate(blocks)], dtype=torch.int32, device=self.kv.device)
        native().kvx_copy_blocks(stage, self.kv.data_ptr(), self.block_bytes, self.layer_block_bytes, pairs,
                                 self._seg_tensors()[0], self.layer_block_bytes, COPY_ENGINE)
        return stage, pairs

    def _unpack(self, stage: torch.Tensor, blocks: list):
        """Scatter slab rows back into the pool blocks (current stream)."""
        n = len(blocks)
        if not self.kv.is_cuda:
            idx = torch.tensor(blocks, dtype=torch.long)
            blk = stage[:n].contiguous().view(self.kv.dtype).view((n,) + self.blk_shape)
            self.kv.index_copy_(1, idx, blk.transpose(0, 1))
            return None
        from llmd_amd.kvx.agent import COPY_ENGINE
        from llmd_amd.ops import native

        pairs = torch.tensor([[j, b] for j, b in enumerate(blocks)], dtype=torch.int32, device=self.kv.device)
        native().kvx_copy_blocks(self.kv, stage.data_ptr(), self.layer_block_bytes, self.block_bytes, pairs,
                                 self._seg_tensors()[1], self.layer_block_bytes, COPY_ENGINE)
        return pairs

    # ------------------------------------------------------------ weight sync / sleep (engine/weight_sync.py)
    def _drain(self):
        """Wait for every copy on the side stream and every FS I/O that reads a host
        slot; commit the write-through copies that landed (their slots hold valid KV)."""
        if self.stream is not None:
            self.stream.synchronize()
        done, self.pending = self.pending, []
        for item in done:
            self._finish_store(item)
        if self.fs is not None:
            self.fs.flush()
            self._poll_fs()

    def invalidate(self, weights_id: str):
        """New weights: every cached block holds KV of the old ones. Drop the host
        tier (removal events for the router's index) and move FS keys to the new
        weights' namespace, so files of the old weights are never read again."""
        self._drain()
        # reloads still in flight carry KV of the old weights: they report 0 tokens (the
        # scheduler recomputes) and give their slot references back before the reset
        self._cancel_inflight_loads()
        for key in list(self.slot_of):
            self.events_out.append((1, key, 0, -1, [], "cpu"))
        self.slot_of.clear()
        self.slot_busy.clear()
        self.free_slots = list(range(self.n_slots - 1, -1, -1))
        self.weights_id = weights_id
        self.ns = self._namespace(weights_id)

    def rebind(self, kv):
        """The device pool is released (``kv=None``, sleep) or was re-allocated
        (wake-up). In-flight D2H copies read the old pool: wait for them (they
        landed, so they are committed to the host tier - their slots are not
        lost) before the pool can be freed; in-flight reloads write into the old
        pool and are finished the same way."""
        self._drain()
        # a reload in flight scattered into the OLD pool (or was never copied when the
        # pool is gone): none of its tokens are resident in the pool used from now on
        self._cancel_inflight_loads()
        self.kv = kv
        if kv is not None:
            self._layout(kv)

    def _cancel_inflight_loads(self):
        """Wait for every reload's FS reads and copies, then make it report 0 tokens
        and release the host slots it holds (poll_loads still returns the request,
        so the scheduler recomputes its prefix instead of trusting the blocks)."""
        if self.fs is not None:
            while any(job.fs_tickets for job in self.loads.values()):
                self.fs.flush()
                self._poll_fs()
        for job in self.loads.values():
            if job.event is not None:
                job.event.synchronize()
            job.n_ok = 0
            self._release_job_slots(job, loaded=False)

    # ------------------------------------------------------------ write-through
    def on_block_events(self, events: list):
        """Engine BlockManager events of the step just executed."""
        todo = [(int(h), int(b)) for kind, h, parent, b, toks in events if kind == 0]
        if not todo or self.kv is None:
            return
        todo = [(h, b) for h, b in todo if h not in self.slot_of]
        if not todo:
            return
        assign = []
        for h, b in todo:
            slot = self._alloc_slot()
            if slot is None:
                break
            assign.append((h, b, slot))
        if not assign:
            return
        blocks = [b for _, b, _ in assign]
        nbytes = len(assign) * self.block_bytes
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record(self.stream)
                stage, pairs = self._pack(blocks)
                packed = torch.cuda.Event()
                packed.record(self.stream)
                for i, s0, r in _slot_runs([slot for _, _, slot in assign]):
                    self.host[s0:s0 + r].copy_(stage[i:i + r], non_blocking=True)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self.stream)
            # a committed block can be released and re-filled by the very next step (the
            # windowed pool recycles blocks every step): that step may write only after the
            # gather read it (the slow D2H copies run on behind)
            torch.cuda.current_stream().wait_event(packed)
            # the staging slab and the pair list stay referenced until the copies land, so the
            # caching allocator cannot hand their memory to the compute stream early
            self.pending.append((ev, [(h, s) for h, _, s in assign], (stage, pairs), ev0, nbytes))
        else:
            t0 = time.perf_counter()
            rows = self._pack(blocks)
            for i, (h, b, slot) in enumerate(assign):
                self.host[slot].copy_(rows[i])
            self.xfer.add("GPU_to_CPU", nbytes, time.perf_counter() - t0)
            self._commit_host([(h, s) for h, _, s in assign])

    def _alloc_slot(self) -> Optional[int]:
        if self.free_slots:
            return self.free_slots.pop()
        for key, slot in self.slot_of.items():  # LRU order, skipping slots in use by I/O
            if not self.slot_busy[slot]:
                del self.slot_of[key]
                self.stats["evicted_cpu"] += 1
                self.events_out.append((1, key, 0, -1, [], "cpu"))
                return slot
        return None

    def _commit_host(self, pairs):
        for h, s in pairs:
            self.slot_of[h] = s
            self.stats["offloaded"] += 1
            self.events_out.append((0, h, 0, -1, [], "cpu"))
            if self.fs is not None:
                t = next(self._ticket)
                self.fs_writes[t] = s
                self.slot_busy[s] += 1
                self.fs.write_async(self._fs_key(h), self.host[s].data_ptr(), self.block_bytes, t)

    def _finish_store(self, item):
        ev, pairs, _keep, ev0, nbytes = item
        self.xfer.add("GPU_to_CPU", nbytes, ev0.elapsed_time(ev) * 1e-3)
        self._commit_host(pairs)

    def _poll_fs(self):
        if self.fs is None:
            return
        for t in self.fs.poll_writes():
            s = self.fs_writes.pop(t, None)
            if s is not None:
                self.slot_busy[s] -= 1
        for t, ok in self.fs.poll_reads():
            job = self._fs_read_job.pop(t, None)
            if job is None:
                continue
            job.fs_tickets.discard(t)
            if not ok:
                k = next((j for j, it in enumerate(job.items) if it[3] == t), len(job.items))
                job.n_ok = k if job.n_ok < 0 else min(job.n_ok, k)
            if not job.fs_tickets:
                self._launch_copy(job)
        w, ws, r, rs = self.fs.io_stats()
        dw, dws, dr, drs = w - self._fs_io0[0], ws - self._fs_io0[1], r - self._fs_io0[2], rs - self._fs_io0[3]
        if dw:
            self.xfer.add("CPU_to_FS", dw, dws)
        if dr:
            self.xfer.add("FS_to_CPU", dr, drs)
        self._fs_io0 = [w, ws, r, rs]

    def poll(self):
        keep = []
        for item in self.pending:
            if item[0].query():
                self._finish_store(item)
            else:
                keep.append(item)
        self.pending = keep
        self._poll_fs()

    # ------------------------------------------------------------ engine hooks
    def before_step(self, so):
        self.poll()

    def after_step(self):
        self.poll()

    def render_metrics(self, model: str) -> bytes:
        """vLLM offloading metrics (vllm:kv_offload_*) plus tier block counters and
        host-tier occupancy."""
        self._poll_fs()
        lab = f'model_name="{model}"'
        st = self.stats
        lines = self.xfer.render(lab)
        lines += ["# HELP vllm:kv_offload_blocks_total KV blocks moved by the offload tiers",
                  "# TYPE vllm:kv_offload_blocks_total counter",
                  f'vllm:kv_offload_blocks_total{{{lab},op="store_cpu"}} {st["offloaded"]}',
                  f'vllm:kv_offload_blocks_total{{{lab},op="load_cpu"}} {st["loaded_cpu"]}',
                  f'vllm:kv_offload_blocks_total{{{lab},op="load_fs"}} {st["loaded_fs"]}',
                  f'vllm:kv_offload_blocks_total{{{lab},op="evict_cpu"}} {st["evicted_cpu"]}',
                  "# HELP vllm:kv_offload_cpu_usage_perc Host-tier slots in use",
                  "# TYPE vllm:kv_offload_cpu_usage_perc gauge",
                  f"vllm:kv_offload_cpu_usage_perc{{{lab}}} {len(self.slot_of) / max(1, self.n_slots):.6f}"]
        return ("\n".join(lines) + "\n").encode()

    def take_events(self) -> list:
        out, self.events_out = self.events_out, []
        return out

    # ------------------------------------------------------------ reload (asynchronous)
    def start_load(self, req, tokens: np.ndarray, cached: int, bm) -> int:
        """Start loading the blocks that continue the request's GPU-cached prefix
        from host / disk. Allocates the destination blocks and returns the number
        of tokens being loaded (0: nothing to load, or the request would not fit
        anyway - it is then not reloaded over and over while it waits). The result
        arrives through ``poll_loads``."""
        if self.kv is None:
            return 0
        bs = bm.block_size
        keys = self.block_keys(req, tokens, bs)
        first = cached // bs
        found = self.lookup_chain(keys, first)
        if not found:
            return 0
        # the reloaded prefix plus the block of the next token must fit in what is free
        # now; otherwise the scheduler would release the blocked request's blocks again
        # before it could run, and reload them on every step
        n = len(found)
        need = -(-min(req.num_tokens, (first + n) * bs + 1) // bs) - bm.num_seq_blocks(req.seq_id)
        if bm.num_free() < need:
            return 0
        if not bm.grow(req.seq_id, (first + n) * bs):
            return 0
        self.launch(req, first, list(bm.block_table(req.seq_id)[first:first + n]), found)
        return n * bs

    @staticmethod
    def block_keys(req, tokens: np.ndarray, bs: int):
        return _rt_loader.rt().hash_blocks(tokens[: max(0, len(tokens) - 1)], bs, req.cache_extra)

    def locate(self, k: int):
        """(tier, key, slot) of one block key in the host / disk tiers, or None."""
        s = self.slot_of.get(k)
        if s is not None:
            return ("cpu", k, s)
        if self.fs is not None and self.fs.exists(self._fs_key(k)):
            return ("fs", k, None)
        return None

    def lookup_chain(self, keys, first: int) -> list:
        """The consecutive run of tier-resident blocks continuing block ``first``."""
        found = []
        for i in range(first, len(keys)):
            it = self.locate(int(keys[i]))
            if it is None:
                break
            found.append(it)
        return found

    def launch(self, req, first: int, dst: list, found: list):
        """Start the reload of ``found`` (locate() results) into pool blocks ``dst``."""
        job = _LoadJob(req, first, dst, [], t0=time.perf_counter())
        # host-tier blocks of the chain are pinned BEFORE any FS block takes a slot, so
        # the slot allocation below cannot evict a block this same reload reads
        for tier, k, s in found:
            if tier == "cpu":
                self.slot_of.move_to_end(k)
                self.slot_busy[s] += 1
        for tier, k, s in found:
            if tier == "cpu":
                job.items.append(("cpu", k, s, None))
                continue
            # an FS block is read into a host-tier slot (the pinned slab allocated once at
            # start-up; no per-block pinned allocation on the engine thread) and joins the
            # host tier once the read succeeded; with every slot busy it is not reloaded
            slot = self._alloc_slot()
            if slot is None:
                break
            self.slot_busy[slot] += 1
            t = next(self._ticket)
            job.fs_tickets.add(t)
            self._fs_read_job[t] = job
            job.items.append(("fs", k, slot, t))
            self.fs.read_async(self._fs_key(k), self.host[slot].data_ptr(), self.block_bytes, t)
        if len(job.items) < len(found):  # the chain is truncated at the first block without a slot
            for tier, k, s in found[len(job.items):]:
                if tier == "cpu":
                    self.slot_busy[s] -= 1
            job.n_ok = len(job.items)
        self.loads[req.request_id] = job
        if not job.fs_tickets:
            self._launch_copy(job)

    def _launch_copy(self, job: _LoadJob):
        n = len(job.items) if job.n_ok < 0 else job.n_ok
        if self.kv is None:  # the pool is released (sleep): nothing can be scattered
            n = 0
        job.n_ok = n
        if n == 0:
            job.event = None
            return
        nbytes = n * self.block_bytes
        slots = [it[2] for it in job.items[:n]]
        if self.stream is None:  # CPU engine: synchronous
            stage = self.host[torch.tensor(slots, dtype=torch.long)]
            self._unpack(stage, job.dst[:n])
            job.event = None
            self.xfer.add("CPU_to_GPU", nbytes, time.perf_counter() - job.t0)
            return
        with torch.cuda.stream(self.stream):
            job.ev0 = torch.cuda.Event(enable_timing=True)
            job.ev0.record(self.stream)
            stage = torch.empty(n, self.block_bytes, dtype=torch.uint8, device=self.kv.device)
            for j, s0, r in _slot_runs(slots):  # one H2D copy per run of consecutive host slots
                stage[j:j + r].copy_(self.host[s0:s0 + r], non_blocking=True)
            # the destination blocks may have been freed by a request whose last step is still
            # on the compute stream: scatter only behind it
            self.stream.wait_stream(torch.cuda.current_stream())
            pairs = self._unpack(stage, job.dst[:n])
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(self.stream)
        job.keep = (stage, pairs)
        job.event = ev

    def poll_loads(self) -> list:
        """Finished reloads: [(request, tokens now resident)]. Aborted requests are
        returned too (the scheduler frees their blocks)."""
        if not self.loads:
            return []
        self._poll_fs()
        out = []
        for rid, job in list(self.loads.items()):
            if job.fs_tickets:
                continue
            if job.event is not None and not job.event.query():
                continue
            del self.loads[rid]
            n = max(0, job.n_ok)
            self._release_job_slots(job, loaded=True)
            for tier, *_ in job.items[:n]:
                self.stats["loaded_cpu" if tier == "cpu" else "loaded_fs"] += 1
            if job.event is not None:
                self.xfer.add("CPU_to_GPU", n * self.block_bytes, job.ev0.elapsed_time(job.event) * 1e-3)
            out.append((job.req, n * self.block_size_of(job)))
        return out

    def _release_job_slots(self, job: _LoadJob, loaded: bool):
        """Drop a reload's host-slot references (once). FS blocks that were read
        successfully (``loaded``, within n_ok) stay in their slot as host-tier
        entries; the other FS slots go back to the free list."""
        if job.released:
            return
        job.released = True
        n = max(0, job.n_ok) if loaded else 0
        for j, (tier, k, s, _t) in enumerate(job.items):
            self.slot_busy[s] -= 1
            if tier != "fs":
                continue
            if j < n and k not in self.slot_of:
                self.slot_of[k] = s
                self.events_out.append((0, k, 0, -1, [], "cpu"))
            else:
                self.free_slots.append(s)

    def block_size_of(self, job) -> int:
        return self.engine.bm.block_size

    def cancel_load(self, request_id: str):
        job = self.loads.get(request_id)
        if job is not None:
            job.aborted = True

    def load_prefix(self, req, tokens: np.ndarray, cached: int, bm) -> int:
        """Synchronous form (tools, tests): start the load and wait for it."""
        n = self.start_load(req, tokens, cached, bm)
        if not n:
            return 0
        job = self.loads[req.request_id]
        while job.fs_tickets:
            self.fs.flush()
            self._poll_fs()
        if job.event is not None:
            job.event.synchronize()
        for r, ntok in self.poll_loads():
            if r is req:
                return ntok
        return 0


class HybridOffload:
    """Tiered offload of a hybrid KV cache (engine/hybrid_kv.py): one
    OffloadManager per pool - the full-attention pool and the windowed pool,
    each with its own host slots and FS keys (``-swa``). Both store
    write-through on their group's BlockStored events. A reload extends a
    prefix to block k only if the full pool's blocks [first, k) are in the tiers
    AND the windowed pool holds (on the GPU, or in its tiers) every block of the
    last window before k; both pools' copies run on the side stream and the
    request continues once both landed. The windowed table is grown with real
    blocks up to k (the ones before the window are released right after the
    load), so a partly failed reload simply reports 0 tokens and the request
    recomputes from its GPU-cached prefix."""

    def __init__(self, cfg, engine):
        r = engine.runner
        fb, sb = r.block_bytes(), r.swa_block_bytes()
        share = fb / (fb + sb)
        self.full = OffloadManager(cfg, engine, "full", share)
        self.swa = OffloadManager(cfg, engine, "swa", 1.0 - share)
        self.engine = engine
        self.window = engine.bm.window
        self.pending: dict[str, dict] = {}  # request id -> {"req", "first", "k", "done": {pool: ntok}}

    # ---- store / housekeeping: both pools
    def on_block_events(self, events: list):
        self.full.on_block_events(events)

    def on_swa_events(self, events: list):
        self.swa.on_block_events(events)

    def before_step(self, so):
        self.full.before_step(so)
        self.swa.before_step(so)

    def after_step(self):
        self.full.after_step()
        self.swa.after_step()

    def take_events(self) -> list:
        self.swa.take_events()  # windowed-pool tier changes are not published (the router indexes full blocks)
        return self.full.take_events()

    def render_metrics(self, model: str) -> bytes:
        return self.full.render_metrics(model)

    def invalidate(self, weights_id: str):
        self.full.invalidate(weights_id)
        self.swa.invalidate(weights_id)

    def rebind(self, kv):
        self.full.rebind(kv)
        self.swa.rebind(None if kv is None else self.engine.runner.kv_swa)

    @property
    def stats(self):
        return self.full.stats

    # ---- reload
    def start_load(self, req, tokens, cached: int, bm) -> int:
        if self.full.kv is None or self.swa.kv is None:
            return 0
        bs = bm.block_size
        keys = OffloadManager.block_keys(req, tokens, bs)
        first = cached // bs
        found = self.full.lookup_chain(keys, first)
        if not found:
            return 0
        swa_tab = bm.block_table_swa(req.seq_id)
        resident = {p for p, b in enumerate(swa_tab) if b}
        k = first + len(found)
        while k > first:  # longest extension whose last window is available for the windowed pool
            lo = max(0, k * bs - self.window + 1) // bs
            need = [p for p in range(lo, k) if p not in resident]
            locs = [self.swa.locate(int(keys[p])) for p in need]
            if all(x is not None for x in locs):
                break
            k -= 1
        if k <= first:
            return 0
        n = k - first
        need_full = -(-min(req.num_tokens, k * bs + 1) // bs) - bm.full.num_seq_blocks(req.seq_id)
        need_swa = -(-min(req.num_tokens, k * bs + 1) // bs) - bm.swa.num_seq_blocks(req.seq_id)
        if bm.full.num_free() < need_full or bm.swa.num_free() < need_swa:
            return 0
        if not bm.grow(req.seq_id, k * bs):
            return 0
        self.full.launch(req, first, list(bm.block_table(req.seq_id)[first:k]), found[:n])
        swa_tab = bm.block_table_swa(req.seq_id)
        self.pending[req.request_id] = {"req": req, "n": n * bs, "ok": True, "wait": {"full"}}
        if need:
            self.swa.launch(req, need[0], [swa_tab[p] for p in need], locs)
            self.pending[req.request_id]["wait"].add("swa")
            self.pending[req.request_id]["swa_n"] = len(need) * bs
        return n * bs

    def poll_loads(self) -> list:
        out = []
        for name, mgr in (("full", self.full), ("swa", self.swa)):
            for req, ntok in mgr.poll_loads():
                st = self.pending.get(req.request_id)
                if st is None:
                    continue
                want = st["n"] if name == "full" else st.get("swa_n", 0)
                st["ok"] = st["ok"] and ntok == want
                st["wait"].discard(name)
        for rid, st in list(self.pending.items()):
            if st["wait"]:
                continue
            del self.pending[rid]
            req = st["req"]
            ntok = st["n"] if st["ok"] else 0
            if ntok and not req.status.finished:
                # blocks before the window of the next query were grown only to keep the
                # table dense: release them now
                self.engine.bm.after_compute(req.seq_id, req.num_computed_tokens + ntok)
            out.append((req, ntok))
        return out

    def cancel_load(self, request_id: str):
        self.full.cancel_load(request_id)
        self.swa.cancel_load(request_id)

    @property
    def loads(self):
        return {**self.swa.loads, **self.full.loads}
