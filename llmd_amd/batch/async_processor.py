"""Async Processor: queue-driven, gated dispatch of individual inference
requests to the router (reference
docs/architecture/advanced/batch/async-processor.md:1-45,
guides/asynchronous-processing/redis/values.yaml).

Roles
* Message queues — ``SortedSetQueue`` (persisted in SQLite, ordered by the
  message deadline: the Redis sorted-set semantics) and ``PubSubQueue``
  (ephemeral, in-process fan-out). Messages are the reference's JSON
  ``{"id", "payload", "deadline"}``; results are appended to a result list.
* Dispatch gates — ``constant`` (always open), ``budget`` (an externally set
  budget value, the ``redis`` gate's role: a file or in-memory key),
  ``prometheus-saturation`` (scrapes the pool's engines ``/metrics`` and opens
  while KV usage and queue depth are below thresholds) and
  ``prometheus-budget`` (free capacity = max_running*pods - running - waiting).
* Workers (default 8) — pull, wait for the gate, dispatch with deadline
  propagation (remaining time -> HTTP timeout), publish results. Retryable
  failures (429/5xx/connection) are re-queued with exponential backoff
  (base 2 s, max 60 s, full jitter); fatal ones (4xx) are not retried;
  requests past their deadline are dropped (``deadline_exceeded``).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import random
import sqlite3
import threading
import time
from typing import Optional

from prometheus_client import CollectorRegistry, Counter, Histogram

log = logging.getLogger("llmd.async")


# ------------------------------------------------------------------ queues
class SortedSetQueue:
    """Persisted priority queue (score = deadline) + result list."""

    def __init__(self, path: str, request_queue: str = "request-sortedset", result_queue: str = "result-list"):
        self.db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self.db.execute("PRAGMA journal_mode=WAL")
        self.db.execute("CREATE TABLE IF NOT EXISTS zset (q TEXT, score REAL, member TEXT, not_before REAL)")
        self.db.execute("CREATE TABLE IF NOT EXISTS list (q TEXT, item TEXT)")
        self.rq, self.resq = request_queue, result_queue
        self.lock = threading.Lock()

    def zadd(self, score: float, member: str, not_before: float = 0.0, queue: Optional[str] = None):
        with self.lock:
            self.db.execute("INSERT INTO zset VALUES (?,?,?,?)", (queue or self.rq, score, member, not_before))

    def pop(self) -> Optional[str]:
        now = time.time()
        with self.lock:
            r = self.db.execute("SELECT rowid, member FROM zset WHERE q=? AND not_before<=? ORDER BY score LIMIT 1",
                                (self.rq, now)).fetchone()
            if r is None:
                return None
            self.db.execute("DELETE FROM zset WHERE rowid=?", (r[0],))
        return r[1]

    def push_result(self, item: str):
        with self.lock:
            self.db.execute("INSERT INTO list VALUES (?,?)", (self.resq, item))

    def rpop_result(self) -> Optional[str]:
        with self.lock:
            r = self.db.execute("SELECT rowid, item FROM list WHERE q=? ORDER BY rowid LIMIT 1",
                                (self.resq,)).fetchone()
            if r is None:
                return None
            self.db.execute("DELETE FROM list WHERE rowid=?", (r[0],))
        return r[1]

    def __len__(self):
        with self.lock:
            return self.db.execute("SELECT COUNT(*) FROM zset WHERE q=?", (self.rq,)).fetchone()[0]


class PubSubQueue:
    """Ephemeral in-process queue (Redis Pub/Sub role): publish / pop; retries
    are delayed in-memory."""

    def __init__(self):
        self.items: list[tuple[float, str]] = []
        self.results: list[str] = []
        self.lock = threading.Lock()

    def zadd(self, score: float, member: str, not_before: float = 0.0, queue=None):
        with self.lock:
            self.items.append((not_before, member))

    publish = zadd

    def pop(self) -> Optional[str]:
        now = time.time()
        with self.lock:
            for i, (nb, m) in enumerate(self.items):
                if nb <= now:
                    del self.items[i]
                    return m
        return None

    def push_result(self, item: str):
        with self.lock:
            self.results.append(item)

    def rpop_result(self) -> Optional[str]:
        with self.lock:
            return self.results.pop(0) if self.results else None

    def __len__(self):
        return len(self.items)


# ------------------------------------------------------------------- gates
class ConstantGate:
    async def budget(self) -> int:
        return 1 << 30


class BudgetGate:
    """External budget: ``value`` set programmatically or read from a file
    (the ``redis`` gate reading a budget key)."""

    def __init__(self, value: int = 0, path: Optional[str] = None):
        self.value, self.path = value, path

    async def budget(self) -> int:
        if self.path and os.path.exists(self.path):
            try:
                with open(self.path) as f:
                    return int(f.read().strip() or 0)
            except (OSError, ValueError):
                return 0
        return self.value


def _parse_prom(text: str) -> dict:
    out = {}
    for line in text.splitlines():
        if not line or line[0] == "#":
            continue
        try:
            name_labels, val = line.rsplit(" ", 1)
            name = name_labels.split("{", 1)[0]
            out[name] = out.get(name, 0.0) + float(val)
        except ValueError:
            continue
    return out


class PrometheusGate:
    """Scrapes engine endpoints' /metrics.
    ``mode='saturation'``: open (budget = free slots) while every scraped pool
    average is below thresholds; ``mode='budget'``: budget = max_running*pods -
    running - waiting."""

    def __init__(self, endpoints: list[str], mode: str = "saturation", kv_threshold: float = 0.8,
                 queue_threshold: float = 5, max_running: int = 64, cache_s: float = 0.05):
        self.endpoints, self.mode = endpoints, mode
        self.kv_threshold, self.queue_threshold = kv_threshold, queue_threshold
        self.max_running, self.cache_s = max_running, cache_s
        self._t, self._val = 0.0, 0
        self._session = None

    async def _scrape(self) -> list[dict]:
        import aiohttp

        if self._session is None:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=2))
        res = []
        for ep in self.endpoints:
            try:
                async with self._session.get(ep.rstrip("/") + "/metrics") as r:
                    res.append(_parse_prom(await r.text()))
            except Exception:  # noqa: BLE001 - unreachable pod counts as saturated
                res.append({"vllm:kv_cache_usage_perc": 1.0, "vllm:num_requests_waiting": 1e9})
        return res

    async def budget(self) -> int:
        now = time.time()
        if now - self._t < self.cache_s:
            return self._val
        ms = await self._scrape()
        running = sum(m.get("vllm:num_requests_running", 0) for m in ms)
        waiting = sum(m.get("vllm:num_requests_waiting", 0) for m in ms)
        if self.mode == "budget":
            val = int(max(0, self.max_running * len(ms) - running - waiting))
        else:
            kv = max((m.get("vllm:kv_cache_usage_perc", 0) for m in ms), default=1.0)
            q = waiting / max(1, len(ms))
            val = int(max(0, self.max_running * len(ms) - running)) if (kv < self.kv_threshold and
                                                                         q < self.queue_threshold) else 0
        self._t, self._val = now, val
        return val

    async def close(self):
        if self._session is not None:
            await self._session.close()


def make_gate(spec: dict):
    t = spec.get("type", "constant")
    if t == "constant":
        return ConstantGate()
    if t in ("redis", "budget"):
        return BudgetGate(int(spec.get("value", 0)), spec.get("path"))
    if t in ("prometheus-saturation", "prometheus-budget"):
        return PrometheusGate(spec.get("endpoints", []), "budget" if t.endswith("budget") else "saturation",
                              float(spec.get("kvThreshold", 0.8)), float(spec.get("queueThreshold", 5)),
                              int(spec.get("maxRunning", 64)))
    raise ValueError(f"unknown gate type {t}")


# --------------------------------------------------------------- processor
class AsyncProcessor:
    BASE_BACKOFF, MAX_BACKOFF = 2.0, 60.0

    def __init__(self, mq, base_url: str, request_path: str = "/v1/completions", gate=None, workers: int = 8,
                 max_retries: int = 10, base_backoff: Optional[float] = None):
        self.mq, self.url = mq, base_url.rstrip("/") + request_path
        self.gate = gate or ConstantGate()
        self.n_workers, self.max_retries = workers, max_retries
        self.base_backoff = self.BASE_BACKOFF if base_backoff is None else base_backoff
        self.inflight = 0
        r = self.registry = CollectorRegistry()
        self.m_total = Counter("async_processor_requests_total", "Requests pulled", registry=r)
        self.m_ok = Counter("async_processor_success_total", "Successful requests", registry=r)
        self.m_fail = Counter("async_processor_failure_total", "Failed requests", registry=r)
        self.m_retry = Counter("async_processor_retries_total", "Retries", registry=r)
        self.m_deadline = Counter("async_processor_deadline_exceeded_total", "Deadline exceeded", registry=r)
        self.m_shed = Counter("async_processor_shedded_total", "Shed by gate until deadline", registry=r)
        self.m_lat = Histogram("async_processor_request_latency_seconds", "Dispatch latency", registry=r)
        self._tasks: list[asyncio.Task] = []
        self._session = None
        self._lock = asyncio.Lock()

    def backoff(self, attempt: int) -> float:
        return random.uniform(0, min(self.MAX_BACKOFF, self.base_backoff * (2 ** attempt)))

    async def start(self):
        import aiohttp

        self._session = aiohttp.ClientSession()
        self._tasks = [asyncio.get_running_loop().create_task(self._worker(i)) for i in range(self.n_workers)]

    async def stop(self):
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        if self._session:
            await self._session.close()

    async def _acquire(self, deadline: float) -> bool:
        while True:
            async with self._lock:
                if self.inflight < await self.gate.budget():
                    self.inflight += 1
                    return True
            if time.time() >= deadline:
                return False
            await asyncio.sleep(0.05)

    async def _worker(self, i: int):
        while True:
            raw = self.mq.pop()
            if raw is None:
                await asyncio.sleep(0.02)
                continue
            try:
                msg = json.loads(raw)
            except json.JSONDecodeError:
                self.m_fail.inc()
                continue
            await self.handle(msg)

    async def handle(self, msg: dict):
        import aiohttp

        self.m_total.inc()
        deadline = float(msg.get("deadline", time.time() + 3600))
        if time.time() >= deadline:
            self.m_deadline.inc()
            self._result(msg, 0, {"error": {"message": "deadline exceeded", "code": "deadline_exceeded"}})
            return
        if not await self._acquire(deadline):
            self.m_shed.inc()
            self._result(msg, 0, {"error": {"message": "deadline exceeded waiting for capacity",
                                            "code": "deadline_exceeded"}})
            return
        t0 = time.time()
        try:
            remaining = max(0.1, deadline - time.time())
            async with self._session.post(self.url, json=msg.get("payload", {}),
                                          headers={"x-request-id": str(msg.get("id", "")),
                                                   "x-llm-d-request-deadline": str(deadline)},
                                          timeout=aiohttp.ClientTimeout(total=remaining)) as r:
                status = r.status
                try:
                    body = await r.json(content_type=None)
                except (ValueError, json.JSONDecodeError):
                    body = {"error": {"message": (await r.text())[:300]}}
        except asyncio.TimeoutError:
            status, body = 0, {"error": {"message": "deadline exceeded", "code": "deadline_exceeded"}}
        except Exception as e:  # noqa: BLE001
            status, body = -1, {"error": {"message": str(e)}}
        finally:
            self.inflight -= 1
        self.m_lat.observe(time.time() - t0)
        if status == 200:
            self.m_ok.inc()
            self._result(msg, 200, body)
            return
        retryable = status in (-1, 429) or status >= 500
        attempt = int(msg.get("attempt", 0))
        if retryable and attempt < self.max_retries:
            delay = self.backoff(attempt)
            if time.time() + delay < deadline:
                self.m_retry.inc()
                m2 = dict(msg, attempt=attempt + 1)
                self.mq.zadd(deadline, json.dumps(m2), not_before=time.time() + delay)
                return
        if status == 0:
            self.m_deadline.inc()
        self.m_fail.inc()
        self._result(msg, status, body)

    def _result(self, msg, status, body):
        self.mq.push_result(json.dumps({"id": msg.get("id"), "status_code": status, "payload": body}))


def main(argv=None):
    p = argparse.ArgumentParser("llmd-async-processor")
    p.add_argument("--igw-base-url", default="http://127.0.0.1:8000")
    p.add_argument("--request-path-url", default="/v1/completions")
    p.add_argument("--message-queue-impl", default="sortedset", choices=["sortedset", "pubsub"])
    p.add_argument("--db", default="/var/lib/llmd-async/mq.db")
    p.add_argument("--request-queue-name", default="request-sortedset")
    p.add_argument("--result-queue-name", default="result-list")
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--gate", default='{"type": "constant"}', help="JSON gate spec")
    a = p.parse_args(argv)
    if a.message_queue_impl == "sortedset":
        os.makedirs(os.path.dirname(a.db) or ".", exist_ok=True)
        mq = SortedSetQueue(a.db, a.request_queue_name, a.result_queue_name)
    else:
        mq = PubSubQueue()
    proc = AsyncProcessor(mq, a.igw_base_url, a.request_path_url, make_gate(json.loads(a.gate)), a.workers)

    async def run():
        await proc.start()
        while True:
            await asyncio.sleep(3600)

    asyncio.run(run())


if __name__ == "__main__":
    main()
