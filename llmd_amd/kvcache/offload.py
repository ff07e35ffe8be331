"""Tiered KV offload: GPU -> pinned host DRAM -> filesystem (SURVEY N14-N16,
C-M15; docs/architecture/advanced/kv-management/kv-offloader.md).

Policy: *write-through*. A block is immutable once full, so as soon as the
engine commits a full block (BlockStored) it is copied D2H on a dedicated
low-priority HIP stream (ordered after the compute stream that produced it)
into a pinned host pool; no copy is ever on the eviction critical path.
The host tier is an LRU over block keys (``cpu_bytes_to_use``); with an FS
tier configured, host-resident blocks are also persisted as one file per block
(``<root>/<key[:2]>/<key>.kv``) by the native C++ thread pool, so KV survives
engine restarts (the llm-d FS connector behaviour).

On admission the scheduler asks ``load_prefix``: blocks continuing the
request's GPU-cached prefix are looked up host-then-disk, copied H2D on the
compute stream (ordered before the forward) into freshly allocated blocks and
committed, so those tokens are skipped by prefill.
Tier changes are published as KV events with ``medium`` cpu / disk so the
router's precise index scores them with tier weights.

The device pool is layer-major ([L, num_blocks, 2, Hkv, bs, D], see
engine/model_runner.py); a host slot holds one block block-major
([L, 2, Hkv, bs, D], ``block_bytes``), so the side stream gathers the step's
blocks into one contiguous staging tensor (one kernel) and DMAs each row to
its slot; reloads DMA a slot into a staging row and scatter it back.
"""
from __future__ import annotations

import collections
import hashlib
import logging
import os
import threading
from typing import Optional

import numpy as np
import torch

from llmd_amd import _rt_loader

log = logging.getLogger("llmd.offload")


class OffloadManager:
    def __init__(self, cfg, engine):
        oc = dict(cfg.kv_offload_config or {})
        extra = oc.get("kv_connector_extra_config", oc)
        self.engine = engine
        self.kv = engine.runner.kv
        self.block_bytes = self.kv[:, 0].numel() * self.kv.element_size()
        self.blk_shape = (self.kv.shape[0],) + tuple(self.kv.shape[2:])  # one block, block-major
        cpu_bytes = int(extra.get("cpu_bytes_to_use", extra.get("cpu_bytes", 1 << 30)))
        self.n_slots = max(1, cpu_bytes // self.block_bytes)
        pin = self.kv.is_cuda
        self.host = torch.empty(self.n_slots, self.block_bytes, dtype=torch.uint8, pin_memory=pin)
        self.slot_of: "collections.OrderedDict[int, int]" = collections.OrderedDict()  # key -> slot (LRU)
        self.free_slots = list(range(self.n_slots - 1, -1, -1))
        self.pending: list = []  # (event, [(key, slot)])
        self.fs = None
        fs = extra.get("fs_root") or next((t.get("root_dir") for t in extra.get("secondary_tiers", [])
                                           if t.get("type") == "fs"), None)
        if fs:
            rt = _rt_loader.rt()
            threads = int(extra.get("n_write_threads", 8))
            self.fs = rt.FsStore(fs, threads)
        self.stream = torch.cuda.Stream(priority=0) if self.kv.is_cuda else None
        self.events_out: list = []
        self.stats = {"offloaded": 0, "loaded_cpu": 0, "loaded_fs": 0, "evicted_cpu": 0}
        self.lock = threading.Lock()
        # FS keys carry a namespace derived from the weights' stable identity
        # (engine/weight_sync.py: checkpoint identity, trainer version or a unique
        # id per update), not a per-process counter: a restarted engine, or another
        # replica sharing fs_root, only ever reads KV computed by the same weights
        self.weights_id = engine.weight_sync.weights_id
        self.ns = self._namespace(self.weights_id)

    @staticmethod
    def _namespace(weights_id: str) -> str:
        return hashlib.sha256(weights_id.encode()).hexdigest()[:12]

    def _fs_key(self, h: int) -> str:
        return f"{h:016x}-{self.ns}"

    # ------------------------------------------------------------ weight sync / sleep (engine/weight_sync.py)
    def invalidate(self, weights_id: str):
        """New weights: every cached block holds KV of the old ones. Drop the host
        tier (removal events for the router's index) and move FS keys to the new
        weights' namespace, so files of the old weights are never read again."""
        if self.stream is not None:
            self.stream.synchronize()
        self.pending = []
        for key in list(self.slot_of):
            self.events_out.append((1, key, 0, -1, [], "cpu"))
        self.slot_of.clear()
        self.free_slots = list(range(self.n_slots - 1, -1, -1))
        self.weights_id = weights_id
        self.ns = self._namespace(weights_id)

    def rebind(self, kv):
        """The device pool is released (``kv=None``, sleep) or was re-allocated
        (wake-up). In-flight D2H copies read the old pool: wait for them, and
        drop their staging tensors, before the pool can be freed. Blocks whose
        copy had not been committed are not published (their KV events were
        never sent)."""
        if self.stream is not None:
            self.stream.synchronize()
        self.pending = []
        self.kv = kv

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
        idx = torch.tensor([b for _, b, _ in assign], dtype=torch.long, device=self.kv.device)
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                g = self.kv.index_select(1, idx).transpose(0, 1).contiguous()  # [n, L, ...] staging
                rows = g.view(len(assign), -1).view(torch.uint8)
                for i, (h, b, slot) in enumerate(assign):
                    self.host[slot].copy_(rows[i], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            # idx (made on the compute stream, read by the side stream's gather) and
            # the staging tensor g stay referenced until the copies land, so the
            # caching allocator cannot hand their memory to the compute stream early
            self.pending.append((ev, [(h, s) for h, _, s in assign], g, idx))
        else:
            rows = self.kv.index_select(1, idx).transpose(0, 1).contiguous().view(len(assign), -1)
            for i, (h, b, slot) in enumerate(assign):
                self.host[slot].copy_(rows[i].view(torch.uint8))
            self._commit_host([(h, s) for h, _, s in assign])

    def _alloc_slot(self) -> Optional[int]:
        if self.free_slots:
            return self.free_slots.pop()
        if not self.slot_of:
            return None
        key, slot = self.slot_of.popitem(last=False)  # LRU victim
        self.stats["evicted_cpu"] += 1
        self.events_out.append((1, key, 0, -1, [], "cpu"))
        return slot

    def _commit_host(self, pairs):
        for h, s in pairs:
            self.slot_of[h] = s
            self.stats["offloaded"] += 1
            self.events_out.append((0, h, 0, -1, [], "cpu"))
            if self.fs is not None:
                self.fs.write(self._fs_key(h), self.host[s].numpy())

    def poll(self):
        keep = []
        for item in self.pending:
            if item[0].query():
                self._commit_host(item[1])
            else:
                keep.append(item)
        self.pending = keep

    # ------------------------------------------------------------ engine hooks
    def before_step(self, so):
        self.poll()

    def after_step(self):
        self.poll()

    def render_metrics(self, model: str) -> bytes:
        """Tier traffic counters (blocks) and host-tier occupancy."""
        lab = f'model_name="{model}"'
        st = self.stats
        lines = ["# HELP llmd:kv_offload_blocks_total KV blocks moved by the offload tiers",
                 "# TYPE llmd:kv_offload_blocks_total counter",
                 f'llmd:kv_offload_blocks_total{{{lab},op="store_cpu"}} {st["offloaded"]}',
                 f'llmd:kv_offload_blocks_total{{{lab},op="load_cpu"}} {st["loaded_cpu"]}',
                 f'llmd:kv_offload_blocks_total{{{lab},op="load_fs"}} {st["loaded_fs"]}',
                 f'llmd:kv_offload_blocks_total{{{lab},op="evict_cpu"}} {st["evicted_cpu"]}',
                 "# HELP llmd:kv_offload_cpu_usage_perc Host-tier slots in use",
                 "# TYPE llmd:kv_offload_cpu_usage_perc gauge",
                 f"llmd:kv_offload_cpu_usage_perc{{{lab}}} {len(self.slot_of) / max(1, self.n_slots):.6f}"]
        return ("\n".join(lines) + "\n").encode()

    def take_events(self) -> list:
        out, self.events_out = self.events_out, []
        return out

    # ------------------------------------------------------------ reload
    def load_prefix(self, req, tokens: np.ndarray, cached: int, bm) -> int:
        """Extend the request's cached prefix from host/disk. Returns the number
        of additional tokens now resident (multiple of block size)."""
        bs = bm.block_size
        rt = _rt_loader.rt()
        keys = rt.hash_blocks(tokens[: max(0, len(tokens) - 1)], bs, req.cache_extra)
        first = cached // bs
        found = []
        for i in range(first, len(keys)):
            k = int(keys[i])
            s = self.slot_of.get(k)
            if s is not None:
                found.append(("cpu", k, s))
                continue
            if self.fs is not None and self.fs.exists(self._fs_key(k)):
                found.append(("fs", k, None))
                continue
            break
        if not found:
            return 0
        n = len(found)
        if not bm.grow(req.seq_id, (first + n) * bs):
            return 0
        table = bm.block_table(req.seq_id)
        stage = torch.empty(n, self.block_bytes, dtype=torch.uint8, device=self.kv.device)
        for j, (tier, k, s) in enumerate(found):
            if tier == "cpu":
                self.slot_of.move_to_end(k)
                stage[j].copy_(self.host[s], non_blocking=True)
                self.stats["loaded_cpu"] += 1
            else:
                buf = torch.empty(self.block_bytes, dtype=torch.uint8, pin_memory=self.kv.is_cuda)
                ok = self.fs.read(self._fs_key(k), buf.numpy())
                if not ok:
                    n = j
                    break
                stage[j].copy_(buf, non_blocking=True)
                self.stats["loaded_fs"] += 1
        if n:
            # scatter the staged block-major rows into the layer-major pool (compute stream, before the forward)
            idx = torch.tensor(table[first:first + n], dtype=torch.long, device=self.kv.device)
            blk = stage[:n].view(self.kv.dtype).view((n,) + self.blk_shape)
            self.kv.index_copy_(1, idx, blk.transpose(0, 1))
        return n * bs
