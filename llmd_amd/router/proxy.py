"""Router data plane: streaming L7 proxy with the EPP in-process (SURVEY C07,
"standalone mode": the reference runs Envoy + ext_proc on localhost; here the
proxy calls the EPP directly and keeps the same contract - the EPP returns
``x-gateway-destination-endpoint`` plus extra upstream headers, responses
stream back *through* the EPP's response hooks).

Failure semantics: InferencePool ``failureMode`` FailOpen (route to a random
healthy endpoint if the EPP itself errors) or FailClose (503);
EPP-generated rejections carry ``x-llm-d-request-dropped-reason``.

High availability (configuration.md:455-459, active-passive): with
``--ha-enable-leader-election`` every replica campaigns for a lease
(llmd_amd.utils.leader); only the leader reports ready on /health and serves
inference, standbys answer 503 until they take over.

CLI (mirrors the EPP flags, guides/no-kubernetes-deployment/README.md:153-190):
  python -m llmd_amd.router.proxy --config-file epp.yaml --endpoints-file endpoints.yaml \
      --port 8081 --metrics-port 9090 --pool-name pool
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import random
import time
from typing import Optional

import aiohttp
from aiohttp import web

from . import headers as H
from .api import ControlPlane
from .datalayer import EndpointStore, FileDiscovery, endpoints_from_yaml
from .epp import EPP, Decision
from ..utils.tracing import inject, span
from .types import SchedulingError

log = logging.getLogger("llmd.router.proxy")

INFERENCE_PATHS = {"/v1/completions", "/v1/chat/completions", "/v1/embeddings", "/v1/responses",
                   "/v1/conversations", "/v1/messages", "/inference/v1/generate",
                   # h2c gRPC (vllmgrpc-parser): through Envoy's ext_proc or router/grpc_proxy.py
                   "/vllm.grpc.engine.VllmEngine/Generate", "/vllm.grpc.engine.VllmEngine/Embed"}
HOP = {"host", "content-length", "transfer-encoding", "connection", "keep-alive"}


class RouterProxy:
    def __init__(self, epp: EPP, failure_mode: str = "FailClose", timeout: float = 1000.0, elector=None):
        self.epp = epp
        self.failure_mode = failure_mode
        self.timeout = timeout
        self.session: Optional[aiohttp.ClientSession] = None
        self.elector = elector  # utils.leader.LeaseElector when HA is on

    @property
    def active(self) -> bool:
        return self.elector is None or self.elector.is_leader

    async def _session(self):
        if self.session is None:
            conn = aiohttp.TCPConnector(limit=40000, keepalive_timeout=90)
            self.session = aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(
                total=self.timeout, sock_connect=5))
        return self.session

    def app(self) -> web.Application:
        app = web.Application(client_max_size=256 * 1024 * 1024)
        app.router.add_route("*", "/metrics", self.metrics)
        app.router.add_get("/health", self.health)
        app.router.add_route("*", "/{tail:.*}", self.handle)
        app.on_startup.append(self._on_start)
        app.on_cleanup.append(self._on_stop)
        return app

    async def _on_start(self, app):
        await self.epp.start()
        if self.elector is not None:
            self.elector.start()

    async def _on_stop(self, app):
        if self.elector is not None:
            self.elector.stop()
        await self.epp.stop()
        if self.session:
            await self.session.close()

    async def metrics(self, req):
        return web.Response(body=self.epp.render_metrics(), content_type="text/plain")

    async def health(self, req):
        if not self.active:
            return web.Response(text="standby", status=503)
        return web.Response(text="ok" if self.epp.store.all() else "no endpoints",
                            status=200 if self.epp.store.all() else 503)

    async def handle(self, req: web.Request):
        path = "/" + req.match_info["tail"]
        if not self.active:
            return web.json_response({"error": {"message": "endpoint picker standby (not the HA leader)"}},
                                     status=503, headers={"x-llm-d-epp-role": "standby"})
        body = await req.read()
        if req.method != "POST" or path not in INFERENCE_PATHS:
            return await self._passthrough(req, path, body)
        with span("gateway.request", {"path": path}, traceparent=req.headers.get("traceparent")):
            try:
                d = await self.epp.handle(path, body, dict(req.headers))
            except SchedulingError as e:
                hdrs = {H.DROPPED_REASON: e.reason} if e.reason else {}
                return web.json_response({"error": {"message": str(e), "code": e.status}}, status=e.status,
                                         headers=hdrs)
            except Exception as e:  # noqa: BLE001 - EPP failure: FailOpen / FailClose
                log.exception("EPP failure")
                eps = self.epp.store.all()
                if self.failure_mode != "FailOpen" or not eps:
                    return web.json_response({"error": {"message": f"endpoint picker failed: {e}"}}, status=503)
                ep = random.choice(eps)
                from .types import InferenceRequest, CIHeaders
                d = Decision(InferenceRequest(path, {}, CIHeaders(dict(req.headers)), len(body)), ep, {})
                d.fail_open = True
            return await self._forward(req, path, body, d)

    async def _passthrough(self, req, path, body):
        eps = self.epp.store.all()
        if not eps:
            return web.json_response({"error": {"message": "no endpoints"}}, status=503)
        ep = random.choice(eps)
        s = await self._session()
        hdrs = {k: v for k, v in req.headers.items() if k.lower() not in HOP}
        async with s.request(req.method, f"http://{ep.key}{path}", data=body or None, headers=hdrs,
                             params=req.query) as r:
            data = await r.read()
            return web.Response(body=data, status=r.status,
                                headers={k: v for k, v in r.headers.items() if k.lower() not in HOP})

    async def _forward(self, req: web.Request, path: str, body: bytes, d: Decision):
        s = await self._session()
        hdrs = {k: v for k, v in req.headers.items() if k.lower() not in HOP}
        hdrs.update(d.headers)
        hdrs[H.REQUEST_ID] = d.req.request_id
        inject(hdrs)
        payload = d.body if d.body is not None else body
        t0 = time.monotonic()
        info = {"ttft": None, "usage": None, "status": None}
        first = None
        last_tok = None
        n_chunks = 0
        try:
            async with s.post(f"http://{d.endpoint.key}{path}", data=payload, headers=hdrs) as r:
                info["status"] = r.status
                out_h = {k: v for k, v in r.headers.items() if k.lower() not in HOP}
                self.epp.on_response_headers(d, r.status, out_h)
                resp = web.StreamResponse(status=r.status, headers=out_h)
                await resp.prepare(req)
                buf = bytearray()  # response tail for the usage block (trimmed in amortised O(1))
                async for chunk in r.content.iter_any():
                    now = time.monotonic()
                    if first is None:
                        first = now
                    last_tok = now
                    n_chunks += 1
                    self.epp.on_response_chunk(d, chunk, now)
                    buf += chunk
                    if len(buf) > 131072:
                        del buf[:-65536]
                    await resp.write(chunk)
                await resp.write_eof()
                info["usage"] = _find_usage(bytes(buf))
                return resp
        except (aiohttp.ClientError, asyncio.TimeoutError) as e:
            info["status"] = 502
            return web.json_response({"error": {"message": f"upstream {d.endpoint.key} failed: {e}"}}, status=502)
        finally:
            end = time.monotonic()
            info["duration"] = end - t0
            if first is not None and (d.req.stream or info["status"] == 200):
                info["ttft"] = first - t0
            usage = info.get("usage") or {}
            n = usage.get("completion_tokens") or 0
            if first is not None and n > 1 and last_tok is not None:
                info["tpot"] = (last_tok - first) / (n - 1)
            if not getattr(d, "fail_open", False):
                self.epp.on_response_complete(d, info)


def _find_usage(buf: bytes, grpc: bool = False) -> Optional[dict]:
    """Usage from the tail of a JSON or SSE response (needs stream_options.include_usage),
    or from the gRPC Generate response frames (``complete`` / counted ``chunk`` tokens)."""
    if grpc:
        from llmd_amd.serving import vllm_grpc as vg

        try:
            return vg.usage_of_responses(vg.unframe(buf))
        except Exception:  # noqa: BLE001 - a partial / foreign stream: no usage
            return None
    txt = buf.decode("utf-8", errors="ignore")
    if txt.lstrip().startswith("{"):
        try:
            return json.loads(txt).get("usage")
        except json.JSONDecodeError:
            pass
    for line in reversed(txt.splitlines()):
        line = line.strip()
        if line.startswith("data:") and "usage" in line:
            try:
                u = json.loads(line[5:].strip()).get("usage")
                if u:
                    return u
            except json.JSONDecodeError:
                continue
    return None


def main(argv=None):
    p = argparse.ArgumentParser("llmd-amd router (proxy + EPP, standalone mode)")
    p.add_argument("--config-file")
    p.add_argument("--config-text")
    p.add_argument("--endpoints-file", help="file-discovery endpoints.yaml")
    p.add_argument("--endpoints", default="", help="comma list ip:port[:role]")
    p.add_argument("--control-plane", help="YAML with InferencePool/Objective/ModelRewrite docs")
    p.add_argument("--pool-name", default="pool")
    p.add_argument("--pool-namespace", default="default")
    p.add_argument("--port", type=int, default=8081)
    p.add_argument("--metrics-port", type=int, default=9090)
    p.add_argument("--failure-mode", default="FailOpen", choices=["FailOpen", "FailClose"])
    p.add_argument("--ha-enable-leader-election", action="store_true",
                   help="active-passive HA: only the lease holder serves")
    p.add_argument("--ha-lease-file", default=None, help="lease record shared by the replicas")
    p.add_argument("--ha-lease-duration", type=float, default=15.0)
    p.add_argument("--ha-renew-deadline", type=float, default=10.0)
    p.add_argument("--ha-retry-period", type=float, default=2.0)
    p.add_argument("--grpc-port", type=int, default=0,
                   help="also serve the vLLM gRPC engine API (h2c) through the EPP on this port")
    p.add_argument("--grpc-upstream-port-offset", type=int, default=0,
                   help="engine gRPC port = endpoint (HTTP) port + offset")
    p.add_argument("--workers", type=int, default=1,
                   help="proxy worker processes (SO_REUSEPORT) in front of one EPP process; 1 = all in-process "
                        "(the reference's --concurrency, guides/no-kubernetes-deployment/README.md:211)")
    p.add_argument("--data-plane", default="native", choices=["native", "python"],
                   help="with --workers > 1: native = one llmd-relay process with that many epoll threads "
                        "(csrc/relay/relay.cpp, the Envoy role), python = aiohttp worker processes")
    p.add_argument("--v", type=int, default=1)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if a.v >= 3 else logging.INFO)
    text = a.config_text or (open(a.config_file).read() if a.config_file else DEFAULT_CONFIG)
    cp = ControlPlane()
    if a.control_plane:
        cp.load_yaml(open(a.control_plane).read())
    store = EndpointStore()
    epp = EPP(text, store, cp, a.pool_name)
    elector = None
    if a.ha_enable_leader_election:
        from llmd_amd.utils.leader import LeaseElector

        elector = LeaseElector(a.ha_lease_file or f"/tmp/llmd-epp-{a.pool_namespace}-{a.pool_name}.lease",
                               lease_duration=a.ha_lease_duration, renew_deadline=a.ha_renew_deadline,
                               retry_period=a.ha_retry_period)
    prox = RouterProxy(epp, a.failure_mode, elector=elector)
    app = prox.app()

    async def seed(app):
        if a.endpoints_file:
            fd = FileDiscovery("file-discovery", {"path": a.endpoints_file, "watchFile": True})
            app["fd"] = fd
            await fd.start_watch(store)
        if a.endpoints:
            eps = []
            for i, item in enumerate(x for x in a.endpoints.split(",") if x):
                parts = item.split(":")
                labels = {"llm-d.ai/role": parts[2]} if len(parts) > 2 else {}
                eps.append({"name": f"ep{i}", "address": parts[0], "port": int(parts[1]), "labels": labels})
            for e in endpoints_from_yaml({"endpoints": eps}):
                await store.add(e)

    if a.workers > 1:
        from .workers import run_multi

        async def seed_multi():
            class _App(dict):
                pass
            await seed(_App())

        run_multi(epp, elector, "0.0.0.0", a.port, a.metrics_port, a.workers, a.failure_mode, seed=seed_multi,
                  grpc_port=a.grpc_port, grpc_offset=a.grpc_upstream_port_offset, data_plane=a.data_plane)
        return

    app.on_startup.insert(0, seed)

    async def run():
        runner = web.AppRunner(app, access_log=None)
        await runner.setup()
        await web.TCPSite(runner, "0.0.0.0", a.port).start()
        mapp = web.Application()
        mapp.router.add_get("/metrics", prox.metrics)
        mr = web.AppRunner(mapp)
        await mr.setup()
        await web.TCPSite(mr, "0.0.0.0", a.metrics_port).start()
        if a.grpc_port:
            from .grpc_proxy import GrpcRouter, offset_target

            await GrpcRouter(epp, offset_target(a.grpc_upstream_port_offset)).start(a.grpc_port)
        log.info("router listening on :%d (metrics :%d)", a.port, a.metrics_port)
        while True:
            await asyncio.sleep(3600)

    asyncio.run(run())


DEFAULT_CONFIG = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: queue-scorer
- type: kv-cache-utilization-scorer
- type: prefix-cache-scorer
- type: no-hit-lru-scorer
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: queue-scorer
    weight: 2
  - pluginRef: kv-cache-utilization-scorer
    weight: 2
  - pluginRef: prefix-cache-scorer
    weight: 3
  - pluginRef: no-hit-lru-scorer
    weight: 2
"""

if __name__ == "__main__":
    main()
