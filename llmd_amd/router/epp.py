"""Endpoint Picker core.

``EPP.handle()`` is the ext_proc-shaped entry point: headers + body in,
destination endpoint + upstream headers (+ possibly rewritten body) out.
Lifecycle per request:
  parse -> model rewrite -> objective/priority -> flow control (or
  saturation shedding) -> data producers -> admitters -> scheduler
  (profile handler: filters -> weighted scorers -> picker per profile)
  -> pre-request hooks -> destination.
Response hooks (headers / chunks / completion) feed in-flight accounting,
latency samples and metrics.
"""
from __future__ import annotations

import asyncio
import functools
import json
import logging
import random
import time
from dataclasses import dataclass, field
from typing import Optional

from . import headers as H
from .api import ControlPlane
from .config import EPPConfig, load_config
from .datalayer import EndpointStore, MetricsDataSource
from .flow_control import DISPATCHED, OUTCOME_HTTP, OUTCOME_REASON, FlowController
from .metrics import EPPMetrics
from ..utils.tracing import span
from .types import Endpoint, InferenceRequest, ProfileRunResult, SchedulingError, SchedulingResult
from .. import _rt_loader

_RT = _rt_loader.rt()
_rand64 = functools.partial(random.getrandbits, 64)  # Python's random: seeding it keeps picks reproducible

log = logging.getLogger("llmd.router.epp")


@dataclass
class Decision:
    req: InferenceRequest
    endpoint: Endpoint
    headers: dict = field(default_factory=dict)
    body: Optional[bytes] = None  # rewritten body (model rewrite), else None
    result: Optional[SchedulingResult] = None


class EPPContext:
    """Shared runtime handed to plugins (ctx)."""

    def __init__(self):
        self.plugins: dict = {}
        self.inflight_tokens: dict = {}
        self.inflight_requests: dict = {}
        self.metrics: Optional[EPPMetrics] = None
        self.store: Optional[EndpointStore] = None


class EPP:
    def __init__(self, config_text, store: Optional[EndpointStore] = None,
                 control: Optional[ControlPlane] = None, pool_name: str = "pool"):
        self.ctx = EPPContext()
        self.cfg: EPPConfig = load_config(config_text, self.ctx)
        self.ctx.plugins = self.cfg.plugins
        self.store = store or EndpointStore()
        self.ctx.store = self.store
        self.control = control or ControlPlane()
        self.metrics = EPPMetrics(pool_name)
        self.ctx.metrics = self.metrics
        self.flow: Optional[FlowController] = None
        self._started = False
        # every plugin that cares about endpoint lifecycle becomes a listener
        for p in list(self.cfg.plugins.values()) + [s for s, _ in self.cfg.data_sources]:
            if hasattr(p, "on_endpoint_added") or hasattr(p, "on_endpoint_removed"):
                if p not in self.store.listeners:
                    self.store.listeners.append(p)
        for src, exs in self.cfg.data_sources:
            if isinstance(src, MetricsDataSource):
                src.extractors = exs
                src.on_update = self._on_metrics

    def _on_metrics(self, ep):
        if self.flow is not None:
            self.flow.notify()

    async def start(self):
        if self._started:
            return
        self._started = True
        for p in self.cfg.plugins.values():
            await p.start()
        for e in list(self.store.endpoints.values()):
            for l in self.store.listeners:
                fn = getattr(l, "on_endpoint_added", None)
                if fn:
                    r = fn(e)
                    if asyncio.iscoroutine(r):
                        await r
        if self.cfg.flow_control_enabled:
            self.flow = FlowController(self.cfg.flow_control or {}, self.cfg.plugins,
                                       self.cfg.saturation_detector, self.store.all, self.metrics)
            self.flow.start()

    async def stop(self):
        if self.flow:
            await self.flow.stop()
        for p in self.cfg.plugins.values():
            await p.stop()
        for s, _ in self.cfg.data_sources:
            await s.stop()

    # ------------------------------------------------------------ request path
    def parse(self, path: str, body: bytes, headers) -> InferenceRequest:
        try:
            req = self.cfg.parser.parse(path, body, headers)
        except ValueError as e:
            raise SchedulingError(400, str(e)) from e
        # model rewrite: header override, else InferenceModelRewrite rules
        hdr = H.lookup(req.headers, H.MODEL_REWRITE)
        if hdr:
            req.target_model = hdr
        else:
            tgt, rule = self.control.rewrite(req.model)
            if rule is not None:
                self.metrics.child(self.metrics.rewrite, rule, req.model, tgt).inc()
            req.target_model = tgt
        req.objective = H.lookup(req.headers, H.OBJECTIVE)
        req.priority = self.control.priority_of(req.objective)
        req.fairness_id = H.lookup(req.headers, H.FAIRNESS_ID) or H.DEFAULT_FAIRNESS_ID
        req.slo_ttft_ms = H.float_header(req.headers, H.SLO_TTFT)
        req.slo_tpot_ms = H.float_header(req.headers, H.SLO_TPOT)
        rid = req.headers.get(H.REQUEST_ID)
        if rid:
            req.request_id = rid
        return req

    async def handle(self, path: str, body: bytes, headers) -> Decision:
        req = self.parse(path, body, headers)
        with span("gateway.request", {"request_id": req.request_id, "model": req.model}):
            return await self.schedule_request(req, body)

    async def schedule_request(self, req: InferenceRequest, body: bytes) -> Decision:
        m = self.metrics
        m.child(m.req_total, req.model, req.target_model, str(req.priority)).inc()
        m.child(m.req_sizes, req.model, req.target_model).observe(req.raw_size)
        try:
            # ---- flow control / saturation shedding
            if self.flow is not None:
                outcome = await self.flow.enqueue_and_wait(req)
                if outcome != DISPATCHED:
                    raise SchedulingError(OUTCOME_HTTP.get(outcome, 500), f"flow control: {outcome}",
                                          OUTCOME_REASON.get(outcome, ""))
            elif req.sheddable:
                sat = self.cfg.saturation_detector.saturation(self.store.all())
                if sat >= 1.0:
                    raise SchedulingError(429, "pool saturated, sheddable request dropped",
                                          H.REJECTED_SATURATED)
            eps = self.store.all()
            if not eps:
                raise SchedulingError(503, "no ready endpoints in the pool")
            # ---- data producers
            for p in self.cfg.producers:
                t0 = time.perf_counter()
                await p.produce(req, eps)
                m.child(m.plugin_dur, "DataProducer", p.plugin_type, p.name).observe(time.perf_counter() - t0)
            # ---- admitters
            for a in self.cfg.admitters:
                rej = a.admit(req, eps)
                if rej is not None:
                    raise SchedulingError(rej[0], f"rejected by {a.name}", rej[1])
            # ---- schedule
            t0 = time.perf_counter()
            result = self.schedule(req, eps)
            m.sched_e2e.observe(time.perf_counter() - t0)
            tgt = result.target
            if tgt is None:
                m.child(m.sched_attempts, "failure", req.target_model, "", "", "").inc()
                raise SchedulingError(503, "no endpoint satisfied the scheduling profiles")
            m.child(m.sched_attempts, "success", req.target_model, tgt.name, tgt.namespace, str(tgt.port)).inc()
            # ---- pre-request hooks
            for p in self.cfg.pre_request:
                p.pre_request(req, result)
            self.ctx.inflight_requests[tgt.key] = self.ctx.inflight_requests.get(tgt.key, 0) + 1
            if "pd_decision" in req.data:
                m.child(m.pd_decisions, req.target_model, req.data["pd_decision"]).inc()
            hdrs = {H.DESTINATION: tgt.key}
            hdrs.update(result.headers)
            hdrs.update(req.data.get("upstream_headers", {}))
            new_body = None
            if (req.target_model and req.target_model != req.model and isinstance(req.body, dict)
                    and not req.data.get("grpc")):
                b = dict(req.body)
                b["model"] = req.target_model
                new_body = json.dumps(b).encode()
            m.child(m.running, req.model).inc()
            return Decision(req, tgt, hdrs, new_body, result)
        except SchedulingError as e:
            m.child(m.req_err, req.model, req.target_model, str(e.status)).inc()
            raise

    def schedule(self, req: InferenceRequest, eps: list[Endpoint]) -> SchedulingResult:
        handler = self.cfg.profile_handler
        results: dict[str, ProfileRunResult] = {}
        for _ in range(8):  # profile handler rounds (decode -> prefill -> encode)
            names = handler.pick_profiles(req, self.cfg.profiles, results)
            if not names:
                break
            for n in names:
                with span("llm_d.epp.scheduler.profile", {"profile": n}):
                    results[n] = self.run_profile(req, self.cfg.profiles[n], eps)
        if not results:
            raise SchedulingError(503, "profile handler selected no profile")
        with span("llm_d.epp.pd.profile_handler.pick", {"profiles": ",".join(results)}):
            return handler.process_results(req, results)

    def run_profile(self, req, prof, eps) -> ProfileRunResult:
        m = self.metrics
        cand = list(eps)
        for f in prof.filters:
            t0 = time.perf_counter()
            cand = f.filter(req, cand)
            m.child(m.plugin_dur, "Filter", f.plugin_type, f.name).observe(time.perf_counter() - t0)
            if not cand:
                return ProfileRunResult([], {})
        keys = [e.key for e in cand]
        cols, ws = [], []
        for s, w in prof.scorers:
            t0 = time.perf_counter()
            vec = getattr(s, "score_vec", None)
            if vec is not None:  # a list aligned with the candidates
                col = vec(req, cand)
            else:
                get = s.score(req, cand).get
                col = [float(get(k) or 0.0) for k in keys]
            m.child(m.plugin_dur, "Scorer", s.plugin_type, s.name).observe(time.perf_counter() - t0)
            cols.append(col)
            ws.append(float(w))
        # clamp to [0, 1], weight, sum, and the stock pickers: one native call (csrc/runtime/epp_score.cpp)
        picker = prof.picker
        kind = getattr(type(picker), "native_kind", None)
        t0 = time.perf_counter()
        if not cols:
            cols = [[0.0] * len(keys)]
            ws = [0.0]
        n_pick = int(picker.p("maxNumOfEndpoints", 1))
        acc, idx = _RT.combine_pick(cols, ws, n_pick if kind is not None else 0, kind or 0, _rand64())
        if kind is not None:
            picked = [cand[i] for i in idx]
        else:
            picked = picker.pick(req, list(zip(cand, acc)))
        m.child(m.plugin_dur, "Picker", picker.plugin_type, picker.name).observe(time.perf_counter() - t0)
        return ProfileRunResult(picked, dict(zip(keys, acc)))

    # ------------------------------------------------------------ response path
    def on_response_headers(self, d: Decision, status: int, headers: dict):
        for p in self.cfg.response_processors:
            p.on_response_headers(d.req, d.endpoint, status, headers)

    def on_response_chunk(self, d: Decision, chunk: bytes, t: float):
        for p in self.cfg.response_processors:
            p.on_response_chunk(d.req, d.endpoint, chunk, t)

    def on_response_complete(self, d: Decision, info: dict):
        m = self.metrics
        req = d.req
        k = d.endpoint.key
        self.ctx.inflight_requests[k] = max(0, self.ctx.inflight_requests.get(k, 0) - 1)
        m.child(m.running, req.model).dec()
        if info.get("duration") is not None:
            m.child(m.duration, req.model, req.target_model).observe(info["duration"])
        if info.get("ttft") is not None:
            m.child(m.ttft, req.model, req.target_model).observe(info["ttft"])
            if req.slo_ttft_ms and info["ttft"] * 1000 > req.slo_ttft_ms:
                m.child(m.slo_viol, req.model, req.target_model, "ttft").inc()
        usage = info.get("usage") or {}
        if usage:
            m.child(m.in_toks, req.model, req.target_model).observe(usage.get("prompt_tokens", 0))
            m.child(m.out_toks, req.model, req.target_model).observe(usage.get("completion_tokens", 0))
            ct = (usage.get("prompt_tokens_details") or {}).get("cached_tokens")
            if ct is not None:
                m.child(m.cached_toks, req.model, req.target_model).observe(ct)
            n = usage.get("completion_tokens", 0)
            if n and info.get("duration"):
                m.child(m.ntpot, req.model, req.target_model).observe(info["duration"] / n)
        if info.get("tpot") is not None and req.slo_tpot_ms and info["tpot"] * 1000 > req.slo_tpot_ms:
            m.child(m.slo_viol, req.model, req.target_model, "tpot").inc()
        for p in self.cfg.response_processors:
            p.on_response_complete(req, d.endpoint, info)
        if self.flow is not None:
            self.flow.notify()

    def render_metrics(self) -> bytes:
        sat = None
        try:
            sat = self.cfg.saturation_detector.saturation(self.store.all())
        except Exception:  # noqa: BLE001
            pass
        self.metrics.pool_update(self.store.all(), sat)
        for p in self.cfg.plugins.values():
            idx = getattr(p, "index", None)
            if idx is not None and hasattr(idx, "size"):
                self.metrics.prefix_size.set(idx.size())
        return self.metrics.render()
