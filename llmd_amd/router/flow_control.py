"""EPP flow control (docs/architecture/core/router/epp/
flow-control.md:21-419, configuration.md:220-310).

Queues keyed by FlowKey = (fairness id, priority). Dispatch is a continuous
loop: strict priority band -> fairness policy (which flow) -> ordering policy
(which item), gated by the saturation detector (head-of-line blocking while
saturated). Capacity limits (global / per band, bytes and requests) reject
with 429; TTL expiry and client cancellation evict with 503; shutdown with
500. Work-conserving: whenever the detector reports capacity, the next item
is released.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import re
import time
from dataclasses import dataclass, field
from typing import Optional

from .plugins.base import FairnessPolicy, OrderingPolicy, SaturationDetector, register
from .types import KV_USAGE, RUNNING, WAITING, InferenceRequest

# ------------------------------------------------------------------ outcomes
DISPATCHED = "Dispatched"
REJECTED_CAPACITY = "RejectedCapacity"   # 429
EVICTED_TTL = "EvictedTTL"               # 503
EVICTED_CANCELLED = "EvictedContextCancelled"  # 503
REJECTED_OTHER = "RejectedOther"         # 500
OUTCOME_HTTP = {REJECTED_CAPACITY: 429, EVICTED_TTL: 503, EVICTED_CANCELLED: 503, REJECTED_OTHER: 500}
OUTCOME_REASON = {REJECTED_CAPACITY: "rejected-saturated", EVICTED_TTL: "rejected-ttl-expired",
                  EVICTED_CANCELLED: "rejected-context-cancelled", REJECTED_OTHER: "rejected-other"}

_QTY = {"": 1, "k": 10**3, "m": 10**6, "g": 10**9, "t": 10**12, "ki": 2**10, "mi": 2**20, "gi": 2**30,
        "ti": 2**40}


def parse_quantity(v) -> int:
    """Kubernetes quantity ("10Gi", "1k", 512) -> int; 0/None = unlimited."""
    if v is None:
        return 0
    if isinstance(v, (int, float)):
        return int(v)
    m = re.fullmatch(r"\s*([0-9.]+)\s*([A-Za-z]*)\s*", str(v))
    if not m:
        raise ValueError(f"bad quantity {v!r}")
    unit = m.group(2).lower()
    if unit not in _QTY:
        raise ValueError(f"bad quantity unit {v!r}")
    return int(float(m.group(1)) * _QTY[unit])


def parse_duration(v) -> float:
    if v is None:
        return 0.0
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    total = 0.0
    for num, unit in re.findall(r"([0-9.]+)(ms|s|m|h)", s):
        total += float(num) * {"ms": 0.001, "s": 1, "m": 60, "h": 3600}[unit]
    return total


# ------------------------------------------------------------------ policies
@register("fcfs-ordering-policy")
class FCFSOrdering(OrderingPolicy):
    def key(self, item):
        return item.enqueue_time


@register("edf-ordering-policy")
class EDFOrdering(OrderingPolicy):
    def key(self, item):
        return item.deadline if item.deadline is not None else float("inf")


@register("slo-deadline-ordering-policy")
class SLODeadlineOrdering(OrderingPolicy):
    """Deadline = arrival + x-llm-d-slo-ttft-ms; no header -> behind all SLO requests."""

    def key(self, item):
        slo = item.req.slo_ttft_ms
        if slo is None:
            return (1, item.enqueue_time)
        return (0, item.req.arrival + slo / 1000.0)


@register("global-strict-fairness-policy")
class GlobalStrictFairness(FairnessPolicy):
    """Ignore flows: the band's single best item by the ordering policy."""

    def pick_flow(self, band):
        best, bk = None, None
        for f in band.flows.values():
            if not f.heap:
                continue
            k = f.heap[0][0]
            if bk is None or k < bk:
                best, bk = f, k
        return best


@register("round-robin-fairness-policy")
class RoundRobinFairness(FairnessPolicy):
    def pick_flow(self, band):
        ids = [fid for fid, f in band.flows.items() if f.heap]
        if not ids:
            return None
        ids.sort()
        last = band.rr_last
        nxt = next((i for i in ids if last is None or i > last), ids[0])
        band.rr_last = nxt
        return band.flows[nxt]


@register("utilization-detector")
class UtilizationDetector(SaturationDetector):
    """Closed loop on telemetry: an endpoint is saturated when its waiting
    queue >= queueDepthThreshold (default 5) or KV usage >= kvCacheUtilThreshold
    (default 0.8); pool saturation = mean over endpoints of a per-endpoint
    score (1.0 saturated). Stale metrics (> metricsStalenessThreshold) count
    as saturated."""

    def saturation(self, eps):
        if not eps:
            return 1.0
        qd = float(self.p("queueDepthThreshold", 5))
        kv = float(self.p("kvCacheUtilThreshold", 0.8))
        stale = float(str(self.p("metricsStalenessThreshold", "200ms")).rstrip("ms") or 200) / 1000.0
        now = time.monotonic()
        tot = 0.0
        for e in eps:
            ts = e.attrs.get("MetricsUpdateTime")
            if ts is not None and now - ts > max(stale, 1.0):
                tot += 1.0
                continue
            s = max(float(e.metric(WAITING, 0)) / qd if qd else 0.0,
                    float(e.metric(KV_USAGE, 0.0)) / kv if kv else 0.0)
            tot += min(s, 1.0)
        return tot / len(eps)


@register("concurrency-detector")
class ConcurrencyDetector(SaturationDetector):
    """Open loop: in-flight requests (router accounting) vs maxConcurrency per
    endpoint (+ headroom fraction for affinity bursting)."""

    def saturation(self, eps):
        if not eps:
            return 1.0
        mc = float(self.p("maxConcurrency", 128))
        head = float(self.p("headroom", 0.0))
        inflight = getattr(self.ctx, "inflight_requests", None) if self.ctx is not None else None
        total = sum((inflight or {}).get(e.key, 0) for e in eps)
        cap = mc * len(eps) * (1.0 + head)
        return total / cap if cap > 0 else 1.0


# ------------------------------------------------------------------ queues
@dataclass(eq=False)
class QueueItem:
    req: InferenceRequest
    size: int
    enqueue_time: float
    deadline: Optional[float]
    fut: asyncio.Future
    seq: int = 0
    removed: bool = False


@dataclass
class Flow:
    fid: str
    heap: list = field(default_factory=list)


@dataclass
class Band:
    priority: int
    max_bytes: int
    max_requests: int
    ordering: OrderingPolicy
    fairness: FairnessPolicy
    flows: dict = field(default_factory=dict)
    bytes: int = 0
    count: int = 0
    rr_last: Optional[str] = None


class FlowController:
    def __init__(self, cfg: dict, plugins: dict, detector: SaturationDetector, endpoints_fn,
                 metrics=None):
        cfg = cfg or {}
        self.plugins = plugins
        self.detector = detector
        self.endpoints_fn = endpoints_fn
        self.metrics = metrics
        self.max_bytes = parse_quantity(cfg.get("maxBytes", 0))
        self.max_requests = parse_quantity(cfg.get("maxRequests", 0))
        self.default_ttl = parse_duration(cfg.get("defaultRequestTTL", 0))
        self.default_band = dict(cfg.get("defaultPriorityBand") or {})
        self.band_cfg = {int(b["priority"]): b for b in (cfg.get("priorityBands") or [])}
        self.bands: dict[int, Band] = {}
        self.total_bytes = 0
        self.total_count = 0
        self._seq = itertools.count()
        self._wake: Optional[asyncio.Event] = None
        self._task: Optional[asyncio.Task] = None
        self.closed = False
        self.saturation_threshold = float(cfg.get("saturationThreshold", 1.0))
        self.poll_interval = parse_duration(cfg.get("dispatchPollInterval", "10ms")) or 0.01

    def _policy(self, ref, default_type):
        if ref and ref in self.plugins:
            return self.plugins[ref]
        from .plugins.base import create

        return create(default_type, default_type, {}, None)

    def band(self, prio: int) -> Band:
        b = self.bands.get(prio)
        if b is None:
            c = dict(self.default_band)
            c.update(self.band_cfg.get(prio, {}))
            b = Band(prio, parse_quantity(c.get("maxBytes", "1Gi")), parse_quantity(c.get("maxRequests", 0)),
                     self._policy(c.get("orderingPolicyRef"), "fcfs-ordering-policy"),
                     self._policy(c.get("fairnessPolicyRef"), "global-strict-fairness-policy"))
            self.bands[prio] = b
        return b

    def start(self):
        self._wake = asyncio.Event()
        self._task = asyncio.get_running_loop().create_task(self._loop())

    async def stop(self):
        self.closed = True
        for b in self.bands.values():
            for f in b.flows.values():
                for _, _, it in f.heap:
                    if not it.fut.done():
                        it.fut.set_result(REJECTED_OTHER)
                f.heap.clear()
        if self._task:
            self._task.cancel()

    def queue_size(self, prio: Optional[int] = None) -> int:
        if prio is None:
            return self.total_count
        b = self.bands.get(prio)
        return b.count if b else 0

    async def enqueue_and_wait(self, req: InferenceRequest) -> str:
        if self.closed:
            return REJECTED_OTHER
        b = self.band(req.priority)
        size = max(1, req.raw_size)
        if ((self.max_requests and self.total_count + 1 > self.max_requests) or
                (self.max_bytes and self.total_bytes + size > self.max_bytes) or
                (b.max_requests and b.count + 1 > b.max_requests) or
                (b.max_bytes and b.bytes + size > b.max_bytes)):
            return REJECTED_CAPACITY
        ttl = self.default_ttl
        deadline = None
        if req.deadline is not None:
            deadline = req.deadline
        elif ttl > 0:
            deadline = time.monotonic() + ttl
        fut = asyncio.get_running_loop().create_future()
        it = QueueItem(req, size, time.monotonic(), deadline, fut, next(self._seq))
        f = b.flows.get(req.fairness_id)
        if f is None:
            f = b.flows[req.fairness_id] = Flow(req.fairness_id)
        heapq.heappush(f.heap, (b.ordering.key(it), it.seq, it))
        b.count += 1
        b.bytes += size
        self.total_count += 1
        self.total_bytes += size
        if self.metrics:
            self.metrics.fc_enqueue(req, self)
        self._wake.set()
        try:
            if deadline is not None:
                out = await asyncio.wait_for(asyncio.shield(fut), max(0.0, deadline - time.monotonic()))
            else:
                out = await fut
        except asyncio.TimeoutError:
            self._remove(b, f, it)
            out = EVICTED_TTL
        except asyncio.CancelledError:
            self._remove(b, f, it)
            if self.metrics:
                self.metrics.fc_done(req, EVICTED_CANCELLED, time.monotonic() - it.enqueue_time, self)
            raise
        if self.metrics:
            self.metrics.fc_done(req, out, time.monotonic() - it.enqueue_time, self)
        return out

    def _remove(self, b: Band, f: Flow, it: QueueItem):
        if it.removed:
            return
        it.removed = True
        for i, e in enumerate(f.heap):
            if e[2] is it:
                f.heap.pop(i)
                heapq.heapify(f.heap)
                break
        b.count -= 1
        b.bytes -= it.size
        self.total_count -= 1
        self.total_bytes -= it.size

    def _next(self) -> Optional[tuple]:
        for prio in sorted(self.bands, reverse=True):  # strict priority: highest first
            b = self.bands[prio]
            if b.count == 0:
                continue
            f = b.fairness.pick_flow(b)
            if f is None or not f.heap:
                continue
            return b, f
        return None

    def saturated(self) -> bool:
        return self.detector.saturation(self.endpoints_fn()) >= self.saturation_threshold

    async def _loop(self):
        while not self.closed:
            nxt = self._next()
            if nxt is None:
                self._wake.clear()
                try:
                    await asyncio.wait_for(self._wake.wait(), 0.5)
                except asyncio.TimeoutError:
                    pass
                continue
            if self.saturated():
                # head-of-line block until capacity (re-check telemetry periodically)
                self._wake.clear()
                try:
                    await asyncio.wait_for(self._wake.wait(), self.poll_interval)
                except asyncio.TimeoutError:
                    pass
                continue
            b, f = nxt
            _, _, it = heapq.heappop(f.heap)
            if it.removed:
                continue
            it.removed = True
            b.count -= 1
            b.bytes -= it.size
            self.total_count -= 1
            self.total_bytes -= it.size
            if not it.fut.done():
                it.fut.set_result(DISPATCHED)
            # yield so the dispatched request can register its in-flight load
            await asyncio.sleep(0)

    def notify(self):
        """Capacity may have changed (response completed / metrics refreshed)."""
        if self._wake is not None:
            self._wake.set()
