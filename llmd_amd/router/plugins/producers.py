"""Data producers (per-request state) and admitters
(docs/architecture/core/router/epp/request-handling.md:51-85,
docs/architecture/advanced/kv-management/{prefix-cache-aware-routing,kv-indexer}.md,
docs/architecture/advanced/latency-predictor.md).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time
from typing import Optional

from llmd_amd import _rt_loader

from ..types import ATTR_VERSION, BLOCK_SIZE, KV_USAGE, NUM_GPU_BLOCKS, RUNNING, WAITING, Endpoint, InferenceRequest
from .base import Admitter, DataProducer, PreRequest, ResponseProcessor, register

log = logging.getLogger("llmd.router.producers")

CHARS_PER_TOKEN = 4


@register("approx-prefix-cache-producer")
class ApproxPrefixCacheProducer(DataProducer, PreRequest):
    """Character-block rolling hash chain + per-server LRU learned on route.
    Params: blockSizeTokens (default 64), maxPrefixBlocksToMatch (256),
    maxPrefixTokensToMatch, lruCapacityPerServer (31250), autoTune (true:
    each server's LRU holds as many producer blocks as its KV pool holds
    tokens - ``vllm:cache_config_info`` num_gpu_blocks x block_size /
    blockSizeTokens - so the index forgets prefixes about when the engine
    evicts them instead of crediting a server with everything ever routed
    to it; configuration.md:380-390, agentic-serving.values.yaml:20-29)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        rt = _rt_loader.rt()
        self.block_tokens = int(self.p("blockSizeTokens", self.p("blockSize", 64)))
        self.max_blocks = int(self.p("maxPrefixBlocksToMatch", 256))
        mt = self.p("maxPrefixTokensToMatch")
        if mt:
            self.max_blocks = max(1, int(mt) // self.block_tokens)
        self.index = rt.ApproxIndex(int(self.p("lruCapacityPerServer", 31250)))
        self.rt = rt
        at = self.p("autoTune", True)
        self.auto_tune = at if isinstance(at, bool) else str(at).lower() == "true"
        self._caps: dict[str, int] = {}
        self._seen: dict[str, tuple] = {}
        self._ver, self._n_eps = -1, -1

    def _tune(self, eps):
        v = ATTR_VERSION[0]
        if v == self._ver and len(eps) == self._n_eps:  # no endpoint attribute written since the last scan
            return
        self._ver, self._n_eps = v, len(eps)
        seen = self._seen
        for e in eps:
            raw = (e.metric(NUM_GPU_BLOCKS, 0), e.metric(BLOCK_SIZE, 0))
            if seen.get(e.key) == raw:  # per request per endpoint: skip unchanged pool sizes
                continue
            seen[e.key] = raw
            nb, bs = int(raw[0] or 0), int(raw[1] or 0)
            if nb <= 0 or bs <= 0:
                continue
            cap = max(1, nb * bs // self.block_tokens)
            if self._caps.get(e.key) != cap:
                self._caps[e.key] = cap
                self.index.set_capacity(e.key, cap)

    def _keys(self, req: InferenceRequest) -> list[int]:
        if req.token_ids:
            ks = self.rt.hash_blocks(req.token_ids, self.block_tokens, 0)
            return list(ks[: self.max_blocks])
        return self.rt.char_block_hashes(req.prompt, self.block_tokens * CHARS_PER_TOKEN, 0, self.max_blocks)

    async def produce(self, req, eps):
        if self.auto_tune:
            self._tune(eps)
        keys = self._keys(req)
        req.data.setdefault("prefix_keys", {})[self.name] = keys
        if not keys:
            req.data.setdefault("prefix_match", {})[self.name] = {e.key: 0.0 for e in eps}
            return
        m = self.index.match(keys, [e.key for e in eps])
        req.data.setdefault("prefix_match", {})[self.name] = {k: v / len(keys) for k, v in m.items()}

    def pre_request(self, req, result):
        keys = req.data.get("prefix_keys", {}).get(self.name)
        if not keys:
            return
        for r in result.profile_results.values():
            for e in r.targets[:1]:
                self.index.insert(e.key, keys)

    def on_endpoint_removed(self, ep: Endpoint):
        self.index.remove_server(ep.key)
        self._caps.pop(ep.key, None)
        self._seen.pop(ep.key, None)


@register("token-producer", "tokenizer")
class TokenProducer(DataProducer):
    """Exact token ids via the engine render endpoints
    (/v1/completions/render, /v1/chat/completions/render). Params:
    vllm.url / renderUrl (default http://localhost:8000), modelName."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        v = self.p("vllm") or {}
        self.url = (v.get("url") if isinstance(v, dict) else None) or self.p("renderUrl") or "http://localhost:8000"
        self.local = self.p("localTokenizer")  # callable injected in tests / in-process render
        self.session = None

    async def produce(self, req, eps):
        if req.token_ids is not None:
            return
        if callable(self.local):
            req.token_ids = self.local(req)
            return
        import aiohttp

        if self.session is None:
            self.session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5))
        chat = "messages" in req.body
        path = "/v1/chat/completions/render" if chat else "/v1/completions/render"
        payload = {"model": self.p("modelName") or req.target_model}
        if chat:
            payload["messages"] = req.body["messages"]
        else:
            payload["prompt"] = req.body.get("prompt", "")
        try:
            async with self.session.post(self.url.rstrip("/") + path, json=payload) as r:
                if r.status == 200:
                    d = await r.json()
                    req.token_ids = d.get("token_ids") or d.get("prompt_token_ids")
        except Exception as e:  # noqa: BLE001 - render outage degrades to approximate
            log.debug("render failed: %s", e)

    async def stop(self):
        if self.session is not None:
            await self.session.close()


@register("precise-prefix-cache-producer")
class PrecisePrefixCacheProducer(DataProducer, PreRequest):
    """KV-event-driven index (C++ KVBlockIndex). Params: tokenProcessorConfig
    .blockSize (must equal the engine --block-size), kvEventsConfig
    {topicFilter, concurrency, discoverPods, podDiscoveryConfig.socketPort,
    zmqEndpoint}, speculativeIndexing, speculativeTTL, indexerConfig
    .tierWeights {gpu: 1.0, cpu: 0.8}."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        rt = _rt_loader.rt()
        self.rt = rt
        tpc = self.p("tokenProcessorConfig") or {}
        self.block_size = int(tpc.get("blockSize", self.p("blockSize", 64)))
        ic = self.p("indexerConfig") or {}
        self.index = rt.KVBlockIndex(int(ic.get("maxKeys", 100_000_000)), int(ic.get("podCacheSize", 10)))
        tw = ic.get("tierWeights") or {"gpu": 1.0, "cpu": 0.8}
        self.tier_w = [float(tw.get("gpu", 1.0)), float(tw.get("cpu", 0.8)), float(tw.get("disk", 0.5))]
        self.spec = bool(self.p("speculativeIndexing", False))
        ttl = str(self.p("speculativeTTL", "2s"))
        self.spec_ttl = float(ttl.rstrip("s")) if ttl.endswith("s") else float(ttl)
        ke = self.p("kvEventsConfig") or {}
        self.topic_filter = ke.get("topicFilter", "kv@")
        self.discover = bool(ke.get("discoverPods", True))
        self.socket_port = int((ke.get("podDiscoveryConfig") or {}).get("socketPort", 5556))
        self.central = ke.get("zmqEndpoint")
        self.subs = {}
        self.events_seen = 0

    def extra_key(self, req) -> int:
        return 0

    def _keys(self, req) -> list[int]:
        if not req.token_ids:
            return []
        return list(self.rt.hash_blocks(req.token_ids, self.block_size, self.extra_key(req)))

    async def produce(self, req, eps):
        keys = self._keys(req)
        req.data.setdefault("prefix_keys", {})[self.name] = keys
        if not keys:
            req.data.setdefault("prefix_match", {})[self.name] = {e.key: 0.0 for e in eps}
            return
        pods = [self.pod_of(e) for e in eps]
        s = self.index.score(keys, pods, self.tier_w, 1.0)
        req.data.setdefault("prefix_match", {})[self.name] = {
            e.key: min(1.0, s.get(p, 0.0) / len(keys)) for e, p in zip(eps, pods)}

    def pre_request(self, req, result):
        if not self.spec:
            return
        keys = req.data.get("prefix_keys", {}).get(self.name)
        if not keys:
            return
        for r in result.profile_results.values():
            for e in r.targets[:1]:
                self.index.add_speculative(self.pod_of(e), keys, self.spec_ttl)

    # --- event ingestion
    @staticmethod
    def pod_of(e: Endpoint) -> str:
        return e.key

    def on_batch(self, topic: str, batch: dict, pod: Optional[str] = None):
        if pod is None:
            # topic kv@<ip>:<port>@<model>
            parts = topic.split("@")
            pod = parts[1] if len(parts) >= 2 else topic
        for ev in batch.get("events", []):
            t = ev.get("type")
            medium = (ev.get("medium") or "gpu").lower()
            if t == "BlockStored":
                self.index.add(pod, [int(h) for h in ev["block_hashes"]], medium)
            elif t == "BlockRemoved":
                self.index.remove(pod, [int(h) for h in ev["block_hashes"]], medium)
            elif t == "AllBlocksCleared":
                self.index.clear_pod(pod)
            self.events_seen += 1

    async def on_endpoint_added(self, ep: Endpoint):
        if not self.discover or ep.key in self.subs:
            return
        from llmd_amd.serving.kv_events import KVEventSubscriber

        port = int(ep.labels.get("llm-d.ai/kv-events-port", self.socket_port))
        pod = self.pod_of(ep)
        sub = KVEventSubscriber(f"tcp://{ep.address}:{port}",
                                lambda topic, b, pod=pod: self.on_batch(topic, b, pod), self.topic_filter)
        self.subs[ep.key] = sub.start()

    async def on_endpoint_removed(self, ep: Endpoint):
        sub = self.subs.pop(ep.key, None)
        if sub is not None:
            await sub.stop()
        self.index.clear_pod(self.pod_of(ep))

    async def stop(self):
        for s in list(self.subs.values()):
            await s.stop()


@register("inflight-load-producer")
class InflightLoadProducer(DataProducer, PreRequest, ResponseProcessor):
    """In-flight requests and tokens per endpoint: ++ in PreRequest, -- at EOS."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.reqs: dict[str, int] = {}
        self.toks: dict[str, int] = {}
        self.assigned: dict[str, list] = {}

    async def produce(self, req, eps):
        req.data["inflight"] = {e.key: (self.reqs.get(e.key, 0), self.toks.get(e.key, 0)) for e in eps}

    def _est(self, req):
        n_in = len(req.token_ids) if req.token_ids else max(1, len(req.prompt) // CHARS_PER_TOKEN)
        n_out = int(req.body.get("max_tokens") or req.body.get("max_completion_tokens") or 16)
        return n_in + n_out

    def pre_request(self, req, result):
        t = self._est(req)
        lst = []
        for r in result.profile_results.values():
            for e in r.targets[:1]:
                self.reqs[e.key] = self.reqs.get(e.key, 0) + 1
                self.toks[e.key] = self.toks.get(e.key, 0) + t
                lst.append(e.key)
        self.assigned[req.request_id] = (lst, t)
        if self.ctx is not None:
            self.ctx.inflight_tokens = self.toks

    def on_response_complete(self, req, ep, info):
        lst, t = self.assigned.pop(req.request_id, ([], 0))
        for k in lst:
            self.reqs[k] = max(0, self.reqs.get(k, 0) - 1)
            self.toks[k] = max(0, self.toks.get(k, 0) - t)


@register("predicted-latency-producer")
class PredictedLatencyProducer(DataProducer, PreRequest, ResponseProcessor):
    """Per-endpoint TTFT/TPOT predictions + SLO headroom; streams training
    samples to the latency predictor (C20, latency-predictor.md:18-52).
    Params: predictionServerURL / trainingServerURL (http; env
    PREDICTION_SERVER_URL / TRAINING_SERVER_URL; with neither the predictor
    runs in-process), streamingMode. Training samples (features of the chosen
    endpoint + the observed TTFT/TPOT) are batched and POSTed to the training
    server's /add_training_data_bulk in the background."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        from llmd_amd.router.predictor import LatencyPredictor

        self.url = (self.p("predictionServerURL") or self.p("predictionServerUrl")
                    or os.environ.get("PREDICTION_SERVER_URL"))
        self.train_url = (self.p("trainingServerURL") or self.p("trainingServerUrl")
                          or os.environ.get("TRAINING_SERVER_URL"))
        self.local = None if self.url else LatencyPredictor(min_samples=int(self.p("minSamples", 50)))
        self.session = None
        self.ctx_reqs: dict[str, dict] = {}
        self.ttft_pred_count = 0
        self.available = True
        self.pending: list[dict] = []     # samples waiting for the training server
        self.flush_every = int(self.p("trainingBatchSize", 8))
        self._flushing = False
        self.samples_sent = 0

    def features(self, req, ep: Endpoint, prefix_hit: float, inflight_tokens: int):
        n_in = len(req.token_ids) if req.token_ids else max(1, len(req.prompt) // CHARS_PER_TOKEN)
        return {"kv_cache_percentage": float(ep.metric(KV_USAGE, 0.0)), "input_token_length": n_in,
                "num_request_waiting": float(ep.metric(WAITING, 0)),
                "num_request_running": float(ep.metric(RUNNING, 0)),
                "prefix_cache_score": prefix_hit, "num_tokens_generated": 0,
                "inflight_input_tokens": inflight_tokens}

    def _sess(self):
        import aiohttp

        if self.session is None:
            self.session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=1))
        return self.session

    async def _predict(self, feats: list[dict]):
        if self.local is not None:
            return self.local.predict(feats)
        async with self._sess().post(self.url.rstrip("/") + "/predict/bulk", json={"requests": feats}) as r:
            r.raise_for_status()
            return (await r.json())["predictions"]

    async def _flush(self):
        if self._flushing or not self.pending or not self.train_url:
            return
        self._flushing = True
        batch, self.pending = self.pending, []
        try:
            async with self._sess().post(self.train_url.rstrip("/") + "/add_training_data_bulk",
                                         json={"entries": batch}) as r:
                r.raise_for_status()
                self.samples_sent += len(batch)
        except Exception as e:  # noqa: BLE001 - training server outage: drop, keep routing
            log.debug("training server unavailable: %s", e)
        finally:
            self._flushing = False

    async def _flush_loop(self):
        while True:
            await asyncio.sleep(float(self.p("trainingFlushIntervalS", 0.5)))
            await self._flush()

    async def start(self):
        if self.train_url:
            self._flush_task = asyncio.get_running_loop().create_task(self._flush_loop())

    async def stop(self):
        t = getattr(self, "_flush_task", None)
        if t is not None:
            t.cancel()
        await self._flush()
        if self.session is not None:
            await self.session.close()

    async def produce(self, req, eps):
        from .scheduling import _prefix_info

        hits = _prefix_info(req, None)
        infl = req.data.get("inflight", {})
        feats = [self.features(req, e, hits.get(e.key, 0.0), infl.get(e.key, (0, 0))[1]) for e in eps]
        # features are kept even without a model: the chosen endpoint's become
        # the training sample that bootstraps the first model
        req.data["latency_features"] = {e.key: f for e, f in zip(eps, feats)}
        try:
            preds = await self._predict(feats)
            self.available = True
        except Exception as e:  # noqa: BLE001 - predictor outage: scorers fall back
            log.debug("predictor unavailable: %s", e)
            self.available = False
            return
        if preds is None:
            return
        out = {}
        for e, f, p in zip(eps, feats, preds):
            ttft, tpot = float(p["ttft_ms"]), float(p["tpot_ms"])
            hr_t = (req.slo_ttft_ms - ttft) if req.slo_ttft_ms else 0.0
            hr_p = (req.slo_tpot_ms - tpot) if req.slo_tpot_ms else 0.0
            out[e.key] = {"ttft_ms": ttft, "tpot_ms": tpot, "headroom": min(hr_t, hr_p), "features": f}
        req.data["predicted_latency"] = out
        self.ttft_pred_count += 1

    def pre_request(self, req, result):
        pred = req.data.get("predicted_latency") or {}
        feats = req.data.get("latency_features") or {}
        t = result.target
        if t is None:
            return
        if t.key in pred:
            self.ctx_reqs[req.request_id] = {"features": pred[t.key]["features"], "pred": pred[t.key]}
            if self.ctx is not None and getattr(self.ctx, "metrics", None) is not None:
                self.ctx.metrics.observe_prediction(req, pred[t.key])
        elif t.key in feats:
            self.ctx_reqs[req.request_id] = {"features": feats[t.key], "pred": None}

    def on_response_complete(self, req, ep, info):
        st = self.ctx_reqs.pop(req.request_id, None)
        if st is None or info.get("ttft") is None:
            return
        ttft_ms = 1000 * info["ttft"]
        tpot_ms = 1000 * info["tpot"] if info.get("tpot") else None
        if self.local is not None:
            self.local.add_sample(st["features"], ttft_ms=ttft_ms, tpot_ms=tpot_ms)
        elif self.train_url:
            self.pending.append(dict(st["features"], actual_ttft_ms=ttft_ms, actual_tpot_ms=tpot_ms))
            if len(self.pending) >= self.flush_every:
                try:
                    asyncio.get_running_loop().create_task(self._flush())
                except RuntimeError:  # no loop (sync caller): the periodic flush sends it
                    pass


@register("latency-slo-admitter")
class LatencySLOAdmitter(Admitter):
    """Reject sheddable (priority < 0) requests when no endpoint is predicted
    to meet the request's SLO."""

    def admit(self, req, eps):
        if not req.sheddable:
            return None
        pred = req.data.get("predicted_latency")
        if not pred:
            return None
        if any(v.get("headroom", 0.0) >= 0 for v in pred.values()):
            return None
        return 429, "rejected-saturated"
