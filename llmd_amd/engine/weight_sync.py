"""RL weight synchronisation and engine sleep / wake-up.

The reference names this only as a proposal: the llm-d-rl rollout controller
does "weight sync coordination" and "engine lifecycle (sleep/wake/pause/
resume)" against vLLM workers, with the weights moving over NCCL/NIXL on a
data plane separate from the HTTP control plane
(proposals/non-kubernetes-mode.md:250-291). Here that data plane is a
stand-alone RCCL process group between a trainer and the engine ranks:

* ``init_group(addr, port, rank_offset, world_size)`` - each engine rank
  joins a TCPStore rendezvous the trainer hosts (trainer = rank 0, TP rank r
  of the replica = ``rank_offset + r``) and builds its own ProcessGroupNCCL
  (RCCL over xGMI on one node) or Gloo (CPU) - the default
  ``torch.distributed`` world of the TP group is not involved, so trainers
  can attach and detach without touching the serving collectives.
* ``update_from_group(metas)`` - for every ``(name, dtype, shape)`` the
  trainer broadcasts the FULL HF-named tensor; each rank keeps its TP shard
  through the loader's placement rules (``models/loader.place``), in place,
  so captured hipGraphs keep pointing at the right memory.
* ``update_from_disk(path)`` - the same from safetensors files.

FP8 (``--quantization fp8``) parameters are updated by dequantising into a
bf16 stage, placing the new slice and re-quantising the whole tensor with
the same per-channel / 128x128-block rule (e4m3 round trips of unchanged
rows are exact: their amax maps to 448 again).

Sleep (level 1: weights to pinned host memory, KV cache dropped; level 2:
weights dropped too - the trainer re-sends them) frees the GPU for a
co-located trainer; wake-up re-allocates, restores, re-binds the KV pool and
re-captures the decode hipGraphs (their pointers moved). Sleeping needs an
idle engine; KV producers (their pool is exported to decoders) cannot sleep.
"""
from __future__ import annotations

import datetime
import hashlib
import logging
import os
import time
import uuid
from typing import Optional

import torch
import torch.distributed as dist

from llmd_amd import ops
from llmd_amd.models.loader import _files, place

log = logging.getLogger("llmd.weight_sync")

_DTYPES = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32,
           "float8_e4m3fn": torch.float8_e4m3fn}


def dtype_of(name: str) -> torch.dtype:
    return _DTYPES[name.replace("torch.", "")]


def new_group(addr: str, port: int, rank: int, world_size: int, backend: str, device=None,
              timeout_s: float = 300.0, name: str = "llmd-weight-sync"):
    """A process group outside the default world (trainer + engine ranks)."""
    to = datetime.timedelta(seconds=timeout_s)
    store = dist.TCPStore(addr, int(port), world_size, is_master=(rank == 0), timeout=to)
    pstore = dist.PrefixStore(name, store)
    if backend == "nccl":
        if device is not None:
            torch.cuda.set_device(device)
        pg = dist.ProcessGroupNCCL(pstore, rank, world_size, to)
    else:
        pg = dist.ProcessGroupGloo(pstore, rank, world_size, to)
    return pg, store


def checkpoint_identity(path: str) -> str:
    """A stable name for the weights in a safetensors checkpoint: file names,
    sizes, mtimes and each file's header (tensor names, dtypes, offsets). Two
    replicas loading the same files agree on it; a re-written checkpoint gets a
    new one. Hashing the payload itself (140 GB for a 70B model) would cost
    more than the load."""
    h = hashlib.sha256()
    for f in _files(path):
        st = os.stat(f)
        h.update(f"{os.path.basename(f)}:{st.st_size}:{st.st_mtime_ns}".encode())
        with open(f, "rb") as fh:
            n = int.from_bytes(fh.read(8), "little")
            h.update(fh.read(min(n, 1 << 24)))
    return "ckpt:" + h.hexdigest()[:20]


def initial_identity(cfg) -> str:
    """Identity of the weights an engine starts with (before any update)."""
    q = cfg.quantization or "none"
    if cfg.load_format == "safetensors" and cfg.weights_path:
        return f"{checkpoint_identity(cfg.weights_path)}:{q}"
    return f"dummy:{cfg.model_config.name}:{cfg.seed}:{cfg.dtype}:{q}"


def broadcast(pg, t: torch.Tensor, root: int = 0):
    o = dist.BroadcastOptions()
    o.rootRank = root
    pg.broadcast([t], o).wait()


class WeightSync:
    """Engine-side weight updates and sleep/wake for one rank's ModelRunner."""

    def __init__(self, runner, broadcast_cmd=None):
        self.runner = runner
        self.broadcast_cmd = broadcast_cmd  # TP driver: forward commands to followers
        self.pg = None
        self._store = None
        self.group_rank = -1
        self.sleeping = 0
        # after a level-2 wake-up the weights are uninitialised storage until an
        # update lands: the engine must not step (engine.step checks this)
        self.weights_pending = False
        self._host: dict[str, torch.Tensor] = {}
        self.version = 0  # per-process update counter (metrics / logs only)
        cfg = getattr(runner, "cfg", None)
        # stable identity of the current weights: the FS KV tier namespaces its
        # keys by it, so KV computed by other weights - in this process, an earlier
        # one, or another replica sharing the directory - is never reloaded
        self.weights_id = initial_identity(cfg) if cfg is not None else "unknown"

    # ------------------------------------------------------------ placement
    def _specs(self) -> dict:
        model = self.runner.model
        owner = {}
        for m in model.modules():
            for attr in ("weight", "w1", "w2"):
                p = getattr(m, attr, None)
                if isinstance(p, torch.Tensor):
                    owner[id(p)] = (m, attr)
        out = {}
        for name, p, kind, extra in model.weight_specs():
            out[name] = (p, kind, extra, owner.get(id(p)))
        return out

    def _load_one(self, specs: dict, name: str, full: torch.Tensor) -> bool:
        key = name if name in specs else "model." + name
        if key not in specs:
            return False
        p, kind, extra, own = specs[key]
        full = full.to(p.device)
        mx = p.dtype == torch.uint8 and p.dim() in (3, 4) and own is not None and hasattr(own[0], own[1] + "_scale")
        if p.dtype != torch.float8_e4m3fn and not mx:
            place(p, full, kind, extra)
            return True
        m, attr = own
        s = getattr(m, attr + "_scale" if attr in ("w1", "w2") else "weight_scale")
        with torch.no_grad():
            if mx:  # MXFP4 experts (K-step major [E, K/128, N, 64] or [E, N, K/2]), E8M0 scales [E, N, K/32]
                k = full.shape[1] if kind == "experts_t" else full.shape[-1]
                std = ops.mxfp4_std_layout(p)
                stage = ops.dequant_mxfp4_weight(std, ops.mxfp4_scales_std_layout(s))[..., :k]
                stage = stage.to(torch.bfloat16).contiguous()
                place(stage, full, kind, extra)
                q, ns = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(stage, 2 * std.shape[-1]))
                if p.dim() == 4:
                    q, ns = ops.mxfp4_kernel_layout(q), ops.mxfp4_scales_kernel_layout(ns)
            elif p.dim() == 3:  # block-fp8 experts [E, N, K(padded to 128 on GPU)], scales [E, N/128, K/128]
                k = full.shape[1] if kind == "experts_t" else full.shape[-1]
                stage = ops.dequant_fp8_block_weight(p, s)[..., :k].to(torch.bfloat16).contiguous()
                place(stage, full, kind, extra)
                q, ns = ops.quant_fp8_block_weight(stage)
                q = ops.pad_fp8_k(q, p.shape[-1])
            else:  # per-output-channel [N, K], scale [1, N]
                stage = (p.float() * s.view(-1, 1)).to(torch.bfloat16)
                place(stage, full, kind, extra)
                q, ns = ops.quant_fp8_weight(stage)
            p.copy_(q)
            s.copy_(ns.view_as(s))
        return True

    def _finish(self, n: int, t0: float, src: str, weights_id: str) -> dict:
        if self.runner.is_gpu:
            torch.cuda.synchronize(self.runner.device)
        self.version += 1
        self.weights_id = weights_id
        self.weights_pending = False
        log.info("weights updated from %s: %d tensors in %.2fs (version %d, id %s)", src, n, time.time() - t0,
                 self.version, weights_id)
        return {"updated": n, "version": self.version, "weights_id": weights_id,
                "seconds": round(time.time() - t0, 3)}

    # ------------------------------------------------------------ commands
    def apply(self, cmd: dict):
        """Entry point on every rank (the driver forwards to TP followers first)."""
        if cmd["op"] == "update_from_group" and self.pg is None:  # refuse before followers block in it
            raise RuntimeError("no weight-sync group: call init_group first")
        if self.broadcast_cmd is not None:
            self.broadcast_cmd({"ws_cmd": cmd})
        op = cmd["op"]
        if op == "init_group":
            return self.init_group(cmd["addr"], cmd["port"], cmd["rank_offset"], cmd["world_size"],
                                   cmd.get("backend"), cmd.get("timeout_s", 300.0))
        if op == "update_from_group":
            return self.update_from_group(cmd["metas"], cmd.get("weights_version"))
        if op == "update_from_disk":
            return self.update_from_disk(cmd["path"], cmd.get("weights_version"))
        if op == "destroy_group":
            return self.destroy_group()
        if op == "sleep":
            return self.sleep(int(cmd.get("level", 1)))
        if op == "wake_up":
            return self.wake_up()
        raise ValueError(f"unknown weight-sync op {op}")

    def init_group(self, addr: str, port: int, rank_offset: int, world_size: int,
                   backend: Optional[str] = None, timeout_s: float = 300.0) -> dict:
        from llmd_amd.parallel.state import get_state

        if self.pg is not None:
            self.destroy_group()
        backend = backend or ("nccl" if self.runner.is_gpu else "gloo")
        self.group_rank = int(rank_offset) + get_state().tp_rank
        self.pg, self._store = new_group(addr, port, self.group_rank, int(world_size), backend,
                                         self.runner.device if self.runner.is_gpu else None, timeout_s)
        log.info("joined weight-sync group %s:%s as rank %d/%d (%s)", addr, port, self.group_rank,
                 world_size, backend)
        return {"rank": self.group_rank, "world_size": int(world_size), "backend": backend}

    def destroy_group(self) -> dict:
        self.pg, self._store, self.group_rank = None, None, -1
        return {"destroyed": True}

    @torch.no_grad()
    def update_from_group(self, metas: list, weights_version: Optional[str] = None) -> dict:
        """metas: [(hf_name, dtype name, shape)], broadcast by group rank 0 in order.
        ``weights_version``: the trainer's name for these weights (e.g. its step);
        without one the update gets a unique id, so its KV is never shared."""
        if self.pg is None:
            raise RuntimeError("no weight-sync group: call init_group first")
        if self.sleeping == 2:
            raise RuntimeError("weights were discarded by sleep(level=2): wake_up first")
        t0 = time.time()
        specs = self._specs()
        dev = self.runner.device if self.runner.is_gpu else torch.device("cpu")
        n = 0
        for name, dt, shape in metas:
            buf = torch.empty(tuple(shape), dtype=dtype_of(dt), device=dev)
            broadcast(self.pg, buf, 0)
            n += self._load_one(specs, name, buf)
        wid = f"trainer:{weights_version}" if weights_version is not None else f"group:{uuid.uuid4().hex}"
        return self._finish(n, t0, "group", self._with_quant(wid))

    @torch.no_grad()
    def update_from_disk(self, path: str, weights_version: Optional[str] = None) -> dict:
        from safetensors import safe_open

        t0 = time.time()
        wid = f"trainer:{weights_version}" if weights_version is not None else checkpoint_identity(path)
        specs = self._specs()
        n = 0
        for f in _files(path):
            with safe_open(f, framework="pt", device="cpu") as fh:
                for name in fh.keys():
                    n += self._load_one(specs, name, fh.get_tensor(name))
        return self._finish(n, t0, path, self._with_quant(wid))

    def _with_quant(self, wid: str) -> str:
        cfg = getattr(self.runner, "cfg", None)
        return f"{wid}:{(cfg.quantization if cfg is not None else None) or 'none'}"

    # ------------------------------------------------------------ sleep / wake
    def _tensors(self):
        r = self.runner
        for name, p in r.model.named_parameters():
            yield name, p
        for name, b in r.model.named_buffers():
            yield name, b

    @torch.no_grad()
    def sleep(self, level: int = 1) -> dict:
        r = self.runner
        if self.sleeping:
            return {"sleeping": self.sleeping}
        if getattr(r, "vmm", None) is not None:
            raise RuntimeError("a KV producer's pool is exported to decoders: it cannot sleep")
        if level not in (1, 2):
            raise ValueError("sleep level must be 1 or 2")
        if r.is_gpu:
            torch.cuda.synchronize(r.device)
        # level 2 drops only what a checkpoint (or the trainer) can restore
        ckpt = {id(p) for _, p, _, _ in r.model.weight_specs()} if level == 2 else set()
        freed = 0
        self._nbytes: dict[str, int] = {}
        seen = set()
        for name, t in self._tensors():
            if t.device.type != "cuda":
                continue
            if id(t) not in ckpt:
                h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                h.copy_(t, non_blocking=True)
                self._host[name] = h
            st = t.untyped_storage()
            if st.data_ptr() not in seen:
                seen.add(st.data_ptr())
                freed += st.nbytes()
            self._nbytes[name] = st.nbytes()
        if r.is_gpu:
            torch.cuda.synchronize(r.device)
            for _, t in self._tensors():
                if t.device.type == "cuda":
                    t.untyped_storage().resize_(0)
            r.graphs.clear()
            r.cgraphs.clear()
            r.dbo_graphs.clear()
            if r.kv is not None:
                freed += r.kv.untyped_storage().nbytes()
            r.kv = None
            r._bind(None)
            torch.cuda.empty_cache()
        self.sleeping = level
        log.info("sleep level %d: released %.2f GiB", level, freed / 2**30)
        return {"sleeping": level, "freed_bytes": int(freed)}

    @torch.no_grad()
    def wake_up(self) -> dict:
        r = self.runner
        if not self.sleeping:
            return {"sleeping": 0}
        t0 = time.time()
        if r.is_gpu:
            for name, t in self._tensors():
                if t.device.type != "cuda":
                    continue
                st = t.untyped_storage()
                if st.nbytes() == 0:  # storages shared by several names are restored once
                    st.resize_(self._nbytes[name])
                if name in self._host:
                    t.copy_(self._host[name], non_blocking=True)
            torch.cuda.synchronize(r.device)
            self._host.clear()
            r.kv = r._alloc_cache(r.num_blocks)
            r.capture_graphs()
        level, self.sleeping = self.sleeping, 0
        if level == 2:  # storage is back but holds garbage until the trainer's update
            self.weights_pending = True
        log.info("woke from level %d in %.2fs", level, time.time() - t0)
        return {"sleeping": 0, "woke_from": level, "weights_pending": self.weights_pending,
                "seconds": round(time.time() - t0, 3)}


# ---------------------------------------------------------------- trainer side
class WeightSender:
    """Trainer side of ``update_from_group``: rank 0 of the weight-sync group.

    Typical RL loop (after each optimizer step)::

        snd = WeightSender("127.0.0.1", 29700, world_size=1 + engine_ranks)
        # concurrently: POST /init_weight_update_group to every engine
        snd.connect()
        metas = snd.metas(state_dict)          # send in the body of POST /update_weights
        snd.send(state_dict)                   # concurrently with that POST
    """

    def __init__(self, addr: str, port: int, world_size: int, backend: str = "gloo", device=None,
                 timeout_s: float = 300.0):
        self.addr, self.port, self.world_size = addr, port, world_size
        self.backend, self.device, self.timeout_s = backend, device, timeout_s
        self.pg = None
        self._store = None

    def connect(self):
        self.pg, self._store = new_group(self.addr, self.port, 0, self.world_size, self.backend, self.device,
                                         self.timeout_s)
        return self

    @staticmethod
    def metas(tensors: dict) -> list:
        return [(k, str(v.dtype).replace("torch.", ""), list(v.shape)) for k, v in tensors.items()]

    def send(self, tensors: dict):
        dev = self.device if self.backend == "nccl" else "cpu"
        for _, v in tensors.items():
            broadcast(self.pg, v.to(dev).contiguous(), 0)
