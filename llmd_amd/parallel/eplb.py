"""Expert-parallel load balancing (EPLB).

Reference flags: ``--enable-eplb --eplb-config '{"window_size":1000,
"step_interval":3000,"num_redundant_experts":32}'`` with the constraint
``(E + redundant) % EP == 0`` (guides/wide-ep-lws/modelserver/gpu/vllm/base/
decode.yaml:114-118, prefill.yaml:61-63).

Design (one node, DP attention + EP MoE):

* Every MoE layer holds ``P = E + R`` *physical* expert slots, ``P / EP`` per
  rank. ``phys_to_log[P]`` says which logical expert a slot serves;
  ``log_to_phys[E, max_rep]`` + ``rep_count[E]`` list the replicas.
* Routing maps each (token, k) choice of a logical expert to one of its
  replicas, spreading tokens round-robin by token index - a pure gather, so
  decode hipGraphs capture it; the tables are updated in place.
* Load: ``index_add_`` of ones at the chosen logical ids into a per-layer
  device counter (capturable). Every ``step_interval`` forwards the counters
  are summed over the EP group, a new placement is planned identically on
  every rank (greedy replication of the hottest experts by load/replica, then
  longest-processing-time packing onto ranks, replicas of one expert spread
  over distinct ranks), and expert weights move with batched point-to-point
  sends/recvs (RCCL peer copies over xGMI; gloo on CPU).
"""
from __future__ import annotations

import heapq
import logging
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

log = logging.getLogger("llmd.eplb")


@dataclass
class EplbConfig:
    enabled: bool = False
    window_size: int = 1000
    step_interval: int = 3000
    num_redundant_experts: int = 0


_cfg = EplbConfig()
_layers: list["EplbLayer"] = []
_steps = 0


def configure(enabled: bool, cfg: Optional[dict] = None):
    global _cfg, _layers, _steps
    c = dict(cfg or {})
    _cfg = EplbConfig(enabled=enabled, window_size=int(c.get("window_size", 1000)),
                      step_interval=int(c.get("step_interval", 3000)),
                      num_redundant_experts=int(c.get("num_redundant_experts", 0)))
    _layers = []
    _steps = 0


def config() -> EplbConfig:
    return _cfg


def plan_placement(load: list[float], P: int, n_ranks: int) -> list[int]:
    """phys_to_log for P slots over n_ranks (P % n_ranks == 0) given per-expert load."""
    E = len(load)
    if P < E or P % n_ranks:
        raise ValueError(f"EPLB needs P >= E and P % EP == 0 (P={P}, E={E}, EP={n_ranks})")
    reps = [1] * E
    heap = [(-(load[e] + 1e-9), e) for e in range(E)]  # max load per replica first
    heapq.heapify(heap)
    for _ in range(P - E):
        _, e = heapq.heappop(heap)
        reps[e] += 1
        heapq.heappush(heap, (-(load[e] + 1e-9) / reps[e], e))
    items = sorted(((load[e] / reps[e], e) for e in range(E) for _ in range(reps[e])), key=lambda t: (-t[0], t[1]))
    cap = P // n_ranks
    rank_load = [0.0] * n_ranks
    slots: list[list[int]] = [[] for _ in range(n_ranks)]
    for w, e in items:
        cands = [r for r in range(n_ranks) if len(slots[r]) < cap]
        fresh = [r for r in cands if e not in slots[r]] or cands
        r = min(fresh, key=lambda r: (rank_load[r], r))
        slots[r].append(e)
        rank_load[r] += w
    return [e for r in range(n_ranks) for e in sorted(slots[r])]


def initial_placement(E: int, P: int) -> list[int]:
    """Identity for the first E slots; redundant slots replicate experts 0..R-1."""
    return list(range(E)) + [i % E for i in range(P - E)]


class EplbLayer:
    """Routing tables + load counter of one MoE layer."""

    def __init__(self, E: int, n_ranks: int, rank: int, device, num_redundant: int):
        self.E, self.n, self.rank = E, n_ranks, rank
        self.P = E + num_redundant
        if self.P % n_ranks:
            raise ValueError(f"(experts {E} + redundant {num_redundant}) % EP {n_ranks} != 0")
        self.P_local = self.P // n_ranks
        self.device = device
        self.max_rep = 1 + num_redundant
        self.phys_to_log = initial_placement(E, self.P)
        self.log_to_phys = torch.zeros(E, self.max_rep, dtype=torch.int32, device=device)
        self.rep_count = torch.ones(E, dtype=torch.int32, device=device)
        self.load = torch.zeros(E, dtype=torch.float32, device=device)
        self._write_tables()
        _layers.append(self)

    def _write_tables(self):
        l2p = [[] for _ in range(self.E)]
        for p, e in enumerate(self.phys_to_log):
            l2p[e].append(p)
        tab = torch.zeros(self.E, self.max_rep, dtype=torch.int32)
        cnt = torch.zeros(self.E, dtype=torch.int32)
        for e, ps in enumerate(l2p):
            for i, p in enumerate(ps[: self.max_rep]):
                tab[e, i] = p
            cnt[e] = max(1, min(len(ps), self.max_rep))
        self.log_to_phys.copy_(tab.to(self.device))
        self.rep_count.copy_(cnt.to(self.device))

    def local_logical(self) -> list[int]:
        lo = self.rank * self.P_local
        return self.phys_to_log[lo:lo + self.P_local]

    def route(self, ids: torch.Tensor) -> torch.Tensor:
        """Logical top-k ids [T, k] -> physical slot ids; records the load."""
        T, k = ids.shape
        valid = ids >= 0
        e = torch.where(valid, ids, torch.zeros_like(ids)).long()
        self.load.index_add_(0, e.flatten(), valid.flatten().to(torch.float32))
        pick = (torch.arange(T, device=ids.device, dtype=torch.int64)[:, None] * k
                + torch.arange(k, device=ids.device, dtype=torch.int64)[None, :])
        rep = pick % self.rep_count[e].long()
        phys = self.log_to_phys[e, rep]
        return torch.where(valid, phys.to(ids.dtype), ids)

    def rebalance(self, params: list[torch.Tensor], group=None) -> list[int]:
        """Re-plan from the accumulated load and move expert weights in place.
        ``params``: the layer's per-physical-slot tensors (first dim P_local)."""
        load = self.load.detach().float().cpu()
        if self.n > 1 and dist.is_initialized():
            dist.all_reduce(load, group=group)
        new = plan_placement(load.tolist(), self.P, self.n)
        old = self.phys_to_log
        self.load.zero_()
        if new == old:
            return new
        _move_experts(old, new, self.rank, self.n, self.P_local, params, group)
        self.phys_to_log = new
        self._write_tables()
        return new


def _move_experts(old: list[int], new: list[int], rank: int, n: int, P_local: int, params, group):
    """Make slot s of every rank hold logical new[s]. Sources: the lowest rank
    hosting that expert in ``old`` (a local copy when it is us)."""
    holders: dict[int, list[int]] = {}
    for p, e in enumerate(old):
        holders.setdefault(e, []).append(p)
    lo = rank * P_local
    snap = [t.detach().clone() for t in params]  # old local contents
    # gloo moves host tensors only: stage device weights through CPU (RCCL peer copies otherwise)
    host = dist.is_initialized() and dist.get_backend(group) == "gloo" and params and params[0].is_cuda
    ops = []
    recv_into = []
    # receives / local copies for our new slots
    for i in range(P_local):
        e = new[lo + i]
        if old[lo + i] == e:
            continue
        src_slot = next((p for p in holders[e] if p // P_local == rank), None)
        if src_slot is not None:
            for t, s in zip(params, snap):
                t[i].copy_(s[src_slot - lo])
            continue
        src_slot = holders[e][0]
        for t in params:
            buf = torch.empty_like(t[i], device="cpu" if host else t.device)
            ops.append(dist.P2POp(dist.irecv, buf, _global(src_slot // P_local, group), group))
            recv_into.append((t, i, buf))
    # sends: for every slot on another rank that needs an expert whose first holder is here
    for s_new, e in enumerate(new):
        r_dst = s_new // P_local
        if r_dst == rank or old[s_new] == e:
            continue
        if any(p // P_local == r_dst for p in holders[e]):
            continue  # the destination copies locally
        src_slot = holders[e][0]
        if src_slot // P_local != rank:
            continue
        for s in snap:
            src = s[src_slot - lo].contiguous()
            ops.append(dist.P2POp(dist.isend, src.cpu() if host else src, _global(r_dst, group), group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for t, i, buf in recv_into:
        t[i].copy_(buf)


def _global(group_rank: int, group) -> int:
    if group is None or not dist.is_initialized():
        return group_rank
    return dist.get_global_rank(group, group_rank)


def on_forward(group=None, params_of=None):
    """Called once per executed forward on every EP rank (real or dummy)."""
    global _steps
    if not _cfg.enabled or not _layers:
        return False
    _steps += 1
    if _steps % max(1, _cfg.step_interval):
        return False
    for layer, params in params_of():
        layer.rebalance(params, group)
    log.info("EPLB rebalanced %d MoE layers at forward %d", len(_layers), _steps)
    return True
