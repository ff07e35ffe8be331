"""Batched prometheus children for per-request / per-token hot paths (EPP
decisions, engine steps): see Deferred."""
from __future__ import annotations

import collections
from bisect import bisect_left


class Deferred:
    """Batched labelled child of a Counter or Histogram. ``inc``/``observe`` only
    append to a deque (~0.1 us); ``flush`` folds the batch into the prometheus
    child: one bisect per observation and one locked ``inc`` per touched bucket,
    instead of prometheus' lock + bucket scan per call (~2.5 us; an EPP decision
    makes ~15 such calls, an engine decode step one per running request). Every
    scrape flushes first (``Flusher``), so the
    exposition is exact; deque appends/pops keep a scrape thread safe."""

    __slots__ = ("c", "ub", "q")

    def __init__(self, c):
        self.c = c
        self.ub = list(getattr(c, "_upper_bounds", ()))
        self.q = collections.deque()

    def observe(self, v):
        self.q.append(v)
        if len(self.q) >= 4096:
            self.flush()

    def inc(self, v=1):
        self.q.append(v)
        if len(self.q) >= 4096:
            self.flush()

    def flush(self):
        # The engine thread (inc/observe at 4096 items) and a /metrics scrape
        # (Flusher.collect on the asyncio thread) can flush at once: pop until
        # empty instead of popping a length read earlier.
        q = self.q
        vals = []
        pop = q.popleft
        try:
            while True:
                vals.append(pop())
        except IndexError:
            pass
        if not vals:
            return
        if not self.ub:  # counter
            self.c.inc(sum(vals))
            return
        cnt = [0] * len(self.ub)
        ub = self.ub
        for v in vals:
            cnt[bisect_left(ub, v)] += 1  # first bound >= v: prometheus' ``v <= bound``
        bk = self.c._buckets
        for i, k in enumerate(cnt):
            if k:
                bk[i].inc(k)
        self.c._sum.inc(sum(vals))


class Flusher:
    """Registered first in a registry: every collect (render, a scrape of the
    registry by anyone) flushes the deferred children before the families are
    read. ``m`` is anything with a ``flush()``."""

    def __init__(self, m):
        self.m = m

    def collect(self):
        self.m.flush()
        return []


__all__ = ["Deferred", "Flusher"]
