"""Data layer: endpoint store, discovery, metrics scraping and extraction
(docs/architecture/core/router/epp/datalayer.md,
guides/no-kubernetes-deployment/router/epp/{config,endpoints}.yaml).

* EndpointStore - the pool; notifies listeners on add/remove (the
  endpoint-notification-source role).
* FileDiscovery - `file-discovery` plugin: endpoints.yaml with literal IPs,
  optional `watchFile` (atomic-rename reload).
* MetricsDataSource + CoreMetricsExtractor - one collector per endpoint
  polling Prometheus `/metrics` (default 50 ms) and mapping engine metric
  names (vLLM / SGLang / TRT-LLM, chosen by `llm-d.ai/engine-type`) to the
  standard attribute keys.
"""
from __future__ import annotations

import asyncio
import logging
import os
import re
import time
from typing import Callable, Optional

import yaml

from .plugins.base import DataSource, Extractor, register
from .types import (ACTIVE_LORAS, BLOCK_SIZE, KV_USAGE, MAX_LORA, METRICS_TS, NUM_GPU_BLOCKS, RUNNING,
                    WAITING, WAITING_LORAS, Endpoint)

log = logging.getLogger("llmd.router.datalayer")

_LINE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{(.*)\})?\s+([-+0-9.eEinfNa]+)')
_LABEL = re.compile(r'([a-zA-Z_][a-zA-Z0-9_]*)="((?:[^"\\]|\\.)*)"')


def parse_prometheus(text: str) -> dict[str, list[tuple[dict, float]]]:
    out: dict[str, list] = {}
    for line in text.splitlines():
        if not line or line[0] == "#":
            continue
        m = _LINE.match(line)
        if not m:
            continue
        name, labels, val = m.group(1), m.group(3), m.group(4)
        try:
            v = float(val)
        except ValueError:
            continue
        lab = dict(_LABEL.findall(labels)) if labels else {}
        out.setdefault(name, []).append((lab, v))
    return out


class EndpointStore:
    def __init__(self):
        self.endpoints: dict[str, Endpoint] = {}
        self.listeners: list = []  # objects with async on_endpoint_added/removed

    def all(self) -> list[Endpoint]:
        return [e for e in self.endpoints.values() if e.healthy]

    async def set(self, eps: list[Endpoint]):
        new = {e.key: e for e in eps}
        for k in list(self.endpoints):
            if k not in new:
                await self.remove(k)
        for k, e in new.items():
            if k in self.endpoints:
                self.endpoints[k].labels = e.labels
                self.endpoints[k].name = e.name
            else:
                await self.add(e)

    async def add(self, e: Endpoint):
        self.endpoints[e.key] = e
        for l in self.listeners:
            fn = getattr(l, "on_endpoint_added", None)
            if fn:
                r = fn(e)
                if asyncio.iscoroutine(r):
                    await r

    async def remove(self, key: str):
        e = self.endpoints.pop(key, None)
        if e is None:
            return
        for l in self.listeners:
            fn = getattr(l, "on_endpoint_removed", None)
            if fn:
                r = fn(e)
                if asyncio.iscoroutine(r):
                    await r


def endpoints_from_yaml(doc) -> list[Endpoint]:
    """endpoints.yaml: {endpoints: [{name, address, port|ports, labels, metricsPort}]}
    (one Endpoint per port: DP multi-port pods become several endpoints)."""
    if isinstance(doc, str):
        doc = yaml.safe_load(doc)
    out = []
    for item in (doc or {}).get("endpoints", []) or []:
        ports = item.get("ports") or [item.get("port", 8000)]
        for i, p in enumerate(ports):
            name = item.get("name", item.get("address"))
            out.append(Endpoint(name=f"{name}" if len(ports) == 1 else f"{name}-rank{i}",
                                address=str(item["address"]), port=int(p),
                                namespace=item.get("namespace", "default"),
                                labels=dict(item.get("labels") or {}),
                                metrics_port=item.get("metricsPort")))
    return out


@register("file-discovery")
class FileDiscovery(DataSource):
    """Params: path, watchFile (bool), pollInterval."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.path = self.p("path")
        self.mtime = None
        self.task = None

    async def load(self, store: EndpointStore):
        if not self.path or not os.path.exists(self.path):
            return
        self.mtime = os.path.getmtime(self.path)
        with open(self.path) as f:
            await store.set(endpoints_from_yaml(f.read()))

    async def start_watch(self, store: EndpointStore):
        await self.load(store)
        if not self.p("watchFile", False):
            return

        async def watch():
            while True:
                await asyncio.sleep(float(self.p("pollInterval", 1.0)))
                try:
                    m = os.path.getmtime(self.path)
                except OSError:
                    continue
                if m != self.mtime:
                    try:
                        await self.load(store)
                    except Exception:  # noqa: BLE001 - keep last good set
                        log.exception("endpoints reload failed")

        self.task = asyncio.get_running_loop().create_task(watch())

    async def stop(self):
        if self.task:
            self.task.cancel()


# engine-type specific metric names -> standard attributes
METRIC_MAPS = {
    "vllm": {WAITING: "vllm:num_requests_waiting", RUNNING: "vllm:num_requests_running",
             KV_USAGE: "vllm:kv_cache_usage_perc", "cache_info": "vllm:cache_config_info",
             "lora_info": "vllm:lora_requests_info"},
    "sglang": {WAITING: "sglang:num_queue_reqs", RUNNING: "sglang:num_running_reqs",
               KV_USAGE: "sglang:token_usage", "cache_info": "sglang:cache_config_info"},
    "trtllm-serve": {WAITING: "trtllm_num_requests_waiting", RUNNING: "trtllm_num_requests_running",
                     KV_USAGE: "trtllm_kv_cache_utilization"},
}


@register("core-metrics-extractor")
class CoreMetricsExtractor(Extractor):
    """Params: engineLabelKey (default llm-d.ai/engine-type), defaultEngine (vllm)."""

    def extract(self, ep: Endpoint, data: dict):
        eng = ep.labels.get(self.p("engineLabelKey", "llm-d.ai/engine-type"), self.p("defaultEngine", "vllm"))
        mp = METRIC_MAPS.get(eng, METRIC_MAPS["vllm"])
        upd = {}
        for attr in (WAITING, RUNNING, KV_USAGE):
            rows = data.get(mp.get(attr, ""), [])
            if rows:
                upd[attr] = sum(v for _, v in rows)
        ci = data.get(mp.get("cache_info", ""), [])
        if ci:
            lab = ci[0][0]
            bs = lab.get("block_size", lab.get("page_size"))
            if bs is not None:
                upd[BLOCK_SIZE] = int(float(bs))
            nb = lab.get("num_gpu_blocks", lab.get("num_pages"))
            if nb is not None and nb != "None":
                upd[NUM_GPU_BLOCKS] = int(float(nb))
        li = data.get(mp.get("lora_info", ""), [])
        if li:
            lab, _ = max(li, key=lambda r: r[1])  # latest timestamp wins
            upd[MAX_LORA] = int(float(lab.get("max_lora", 0) or 0))
            upd[ACTIVE_LORAS] = {s.strip() for s in lab.get("running_lora_adapters", "").split(",") if s.strip()}
            upd[WAITING_LORAS] = {s.strip() for s in lab.get("waiting_lora_adapters", "").split(",") if s.strip()}
        upd[METRICS_TS] = time.monotonic()
        ep.attrs.update(upd)


@register("metrics-data-source")
class MetricsDataSource(DataSource):
    """One collector task per endpoint polling http://ep:port/metrics.
    Params: interval (default 50ms), timeout, path."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        from .flow_control import parse_duration

        self.interval = parse_duration(self.p("interval", self.p("refreshMetricsInterval", "50ms"))) or 0.05
        self.timeout = parse_duration(self.p("timeout", "1s")) or 1.0
        self.path = self.p("path", "/metrics")
        self.extractors: list[Extractor] = []
        self.tasks: dict[str, asyncio.Task] = {}
        self.session = None
        self.on_update: Optional[Callable] = None
        self.fetch_override = None  # tests: callable(ep) -> text

    async def on_endpoint_added(self, ep: Endpoint):
        if ep.key not in self.tasks:
            self.tasks[ep.key] = asyncio.get_running_loop().create_task(self._collect(ep))

    async def on_endpoint_removed(self, ep: Endpoint):
        t = self.tasks.pop(ep.key, None)
        if t:
            t.cancel()

    async def _fetch(self, ep: Endpoint) -> Optional[str]:
        if self.fetch_override is not None:
            r = self.fetch_override(ep)
            return await r if asyncio.iscoroutine(r) else r
        import aiohttp

        if self.session is None:
            self.session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout))
        url = f"http://{ep.address}:{ep.metrics_port or ep.port}{self.path}"
        async with self.session.get(url) as r:
            if r.status != 200:
                return None
            return await r.text()

    async def scrape_once(self, ep: Endpoint):
        try:
            text = await self._fetch(ep)
        except Exception:  # noqa: BLE001 - endpoint down: keep stale attrs (staleness detectors see age)
            return
        if text is None:
            return
        data = parse_prometheus(text)
        for x in self.extractors:
            x.extract(ep, data)
        if self.on_update:
            self.on_update(ep)

    async def _collect(self, ep: Endpoint):
        while True:
            await self.scrape_once(ep)
            await asyncio.sleep(self.interval)

    async def stop(self):
        for t in self.tasks.values():
            t.cancel()
        if self.session is not None:
            await self.session.close()


@register("endpoint-notification-source")
class EndpointNotificationSource(DataSource):
    """Marker source: endpoint lifecycle events are delivered to every plugin
    implementing on_endpoint_added / on_endpoint_removed."""
