"""P/D routing sidecar (docs/architecture/advanced/disaggregation/
README.md:104-131, guides/recipes/modelserver/base/single-host/pd/*/patch-sidecar.yaml).

Runs next to a decode engine: clients hit ``--port`` (8000), the local engine
listens on ``--vllm-port`` (8200). For completion requests carrying
``x-prefiller-host-port`` the sidecar drives the KV-transfer protocol:

* ``nixlv2`` (default, two-phase): POST the request to the prefiller with
  ``kv_transfer_params{do_remote_decode: true}``, ``max_tokens=1`` and no
  streaming; take the ``kv_transfer_params`` of its response and POST the
  original request to the local decoder with them (the decoder then pulls
  the KV over kvx). Prefiller 5xx / connection failure -> decode-only
  fallback; prefiller 4xx -> returned to the client (not retried).
* ``sglang``: inject ``bootstrap_host/port/room`` into both requests, fire
  the prefill concurrently, run the decode synchronously.

Multiple prefillers in the header: first one, or a random one with
``--enable-prefiller-sampling``. ``--allowed-prefill-hosts`` (CIDR/host list)
guards against SSRF through the header. ``--data-parallel-size N`` serves
ports port..port+N-1 -> vllm-port..vllm-port+N-1. Other paths pass through.
"""
from __future__ import annotations

import argparse
import asyncio
import copy
import ipaddress
import json
import logging
import random
import time
from typing import Optional

import aiohttp
from aiohttp import web
from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

from llmd_amd.router import headers as H
from llmd_amd.utils.tracing import inject, span

log = logging.getLogger("llmd.sidecar")
COMPLETION_PATHS = {"/v1/completions", "/v1/chat/completions"}
HOP = {"host", "content-length", "transfer-encoding", "connection", "keep-alive"}


class RoutingSidecar:
    def __init__(self, decoder_url: str, connector: str = "nixlv2", prefiller_sampling: bool = False,
                 allowed_hosts: Optional[list[str]] = None, timeout: float = 1000.0,
                 bootstrap_port: int = 8998, secure_prefill: bool = False):
        self.decoder = decoder_url.rstrip("/")
        self.connector = connector
        self.sampling = prefiller_sampling
        self.allowed = [ipaddress.ip_network(a, strict=False) if "/" in a or _is_ip(a) else a
                        for a in (allowed_hosts or [])]
        self.timeout = timeout
        self.bootstrap_port = bootstrap_port
        self.scheme = "https" if secure_prefill else "http"
        self.session: Optional[aiohttp.ClientSession] = None
        r = self.reg = CollectorRegistry()
        self.m_req = Counter("llm_d_pd_proxy_requests", "Requests by path type", ["type"], registry=r)
        self.m_fallback = Counter("llm_d_pd_proxy_prefill_fallbacks", "Decode-only fallbacks", ["reason"],
                                  registry=r)
        self.m_prefill = Histogram("llm_d_pd_proxy_prefill_duration_seconds", "Remote prefill latency",
                                   buckets=(.01, .05, .1, .25, .5, 1, 2, 5, 10, 30, 60), registry=r)
        self.m_ttft = Histogram("llm_d_pd_proxy_true_ttft_seconds", "Client-observed TTFT at the coordinator",
                                buckets=(.01, .05, .1, .25, .5, 1, 2, 5, 10, 30, 60), registry=r)

    async def _s(self):
        if self.session is None:
            self.session = aiohttp.ClientSession(
                connector=aiohttp.TCPConnector(limit=4096, keepalive_timeout=90),
                timeout=aiohttp.ClientTimeout(total=self.timeout, sock_connect=5))
        return self.session

    def app(self) -> web.Application:
        app = web.Application(client_max_size=256 * 1024 * 1024)
        app.router.add_get("/metrics/sidecar", self.metrics)
        app.router.add_route("*", "/{tail:.*}", self.handle)

        async def close(_):
            if self.session:
                await self.session.close()

        app.on_cleanup.append(close)
        return app

    async def metrics(self, req):
        return web.Response(body=generate_latest(self.reg), content_type="text/plain")

    def _allowed(self, hostport: str) -> bool:
        if not self.allowed:
            return True
        host = hostport.rsplit(":", 1)[0].strip("[]")
        for a in self.allowed:
            if isinstance(a, str):
                if a == host:
                    return True
            else:
                try:
                    if ipaddress.ip_address(host) in a:
                        return True
                except ValueError:
                    pass
        return False

    def _pick_prefiller(self, req: web.Request) -> Optional[str]:
        vals = []
        for v in req.headers.getall(H.PREFILLER, []):
            vals.extend(x.strip() for x in v.split(",") if x.strip())
        if not vals:
            return None
        return random.choice(vals) if self.sampling else vals[0]

    async def handle(self, req: web.Request):
        path = "/" + req.match_info["tail"]
        body = await req.read()
        if req.method != "POST" or path not in COMPLETION_PATHS:
            self.m_req.labels("passthrough").inc()
            return await self._proxy(req, self.decoder + path, body, stream_back=True)
        pf = self._pick_prefiller(req)
        if pf is None:
            self.m_req.labels("decode-only").inc()
            return await self._proxy(req, self.decoder + path, body, stream_back=True)
        if not self._allowed(pf):
            return web.json_response({"error": {"message": f"prefiller {pf} not allowed"}}, status=403)
        try:
            data = json.loads(body)
        except json.JSONDecodeError:
            return web.json_response({"error": {"message": "invalid JSON"}}, status=400)
        self.m_req.labels("pd").inc()
        with span("llm_d.pd_proxy.request", {"prefiller": pf, "connector": self.connector},
                  traceparent=req.headers.get("traceparent")):
            if self.connector == "sglang":
                return await self._sglang(req, path, data, pf)
            return await self._nixl(req, path, data, pf)

    async def _nixl(self, req, path, data, pf):
        pre = copy.deepcopy(data)
        pre["kv_transfer_params"] = {"do_remote_decode": True, "do_remote_prefill": False,
                                     "remote_engine_id": None, "remote_block_ids": None,
                                     "remote_host": None, "remote_port": None}
        pre["max_tokens"] = 1
        if "max_completion_tokens" in pre:
            pre["max_completion_tokens"] = 1
        pre["stream"] = False
        pre.pop("stream_options", None)
        hdrs = self._fwd_headers(req)
        t0 = time.monotonic()
        s = await self._s()
        ktp = None
        with span("llm_d.pd_proxy.prefill", {"prefiller": pf}):
            try:
                async with s.post(f"{self.scheme}://{pf}{path}", json=pre, headers=inject(dict(hdrs))) as r:
                    if r.status >= 500:
                        self.m_fallback.labels(f"prefill_{r.status}").inc()
                        log.warning("prefiller %s returned %d: decode-only fallback", pf, r.status)
                    elif r.status >= 400:
                        return web.Response(body=await r.read(), status=r.status,
                                            content_type=r.content_type)
                    else:
                        ktp = (await r.json()).get("kv_transfer_params")
            except (aiohttp.ClientError, asyncio.TimeoutError) as e:
                self.m_fallback.labels("prefill_unreachable").inc()
                log.warning("prefiller %s unreachable (%s): decode-only fallback", pf, e)
        self.m_prefill.observe(time.monotonic() - t0)
        dec = dict(data)
        if ktp:
            dec["kv_transfer_params"] = ktp
        with span("llm_d.pd_proxy.decode", {}):
            return await self._proxy(req, self.decoder + path, json.dumps(dec).encode(), stream_back=True,
                                     t_start=req.get("t0", t0))

    async def _sglang(self, req, path, data, pf):
        room = random.getrandbits(63)
        host = pf.rsplit(":", 1)[0]
        boot = {"bootstrap_host": host, "bootstrap_port": self.bootstrap_port, "bootstrap_room": room}
        pre = dict(data, **boot)
        pre["stream"] = False
        pre.pop("stream_options", None)
        dec = dict(data, **boot)
        s = await self._s()

        async def fire():
            with span("llm_d.pd_proxy.prefill", {"prefiller": pf}):
                try:
                    async with s.post(f"{self.scheme}://{pf}{path}", json=pre,
                                      headers=inject(self._fwd_headers(req))) as r:
                        await r.read()
                except (aiohttp.ClientError, asyncio.TimeoutError) as e:
                    log.warning("sglang prefill to %s failed: %s", pf, e)

        asyncio.get_running_loop().create_task(fire())  # not cancelled with the client
        with span("llm_d.pd_proxy.decode", {}):
            return await self._proxy(req, self.decoder + path, json.dumps(dec).encode(), stream_back=True)

    def _fwd_headers(self, req):
        return {k: v for k, v in req.headers.items()
                if k.lower() not in HOP and k.lower() != H.PREFILLER}

    async def _proxy(self, req, url, body, stream_back=True, t_start=None):
        s = await self._s()
        hdrs = inject(self._fwd_headers(req))
        t0 = t_start or time.monotonic()
        try:
            async with s.request(req.method, url, data=body or None, headers=hdrs, params=req.query) as r:
                resp = web.StreamResponse(status=r.status,
                                          headers={k: v for k, v in r.headers.items() if k.lower() not in HOP})
                await resp.prepare(req)
                first = True
                async for chunk in r.content.iter_any():
                    if first:
                        self.m_ttft.observe(time.monotonic() - t0)
                        first = False
                    await resp.write(chunk)
                await resp.write_eof()
                return resp
        except (aiohttp.ClientError, asyncio.TimeoutError) as e:
            return web.json_response({"error": {"message": f"decoder unavailable: {e}"}}, status=502)


def _is_ip(a: str) -> bool:
    try:
        ipaddress.ip_address(a)
        return True
    except ValueError:
        return False


def main(argv=None):
    p = argparse.ArgumentParser("llmd-amd routing sidecar")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--vllm-port", type=int, default=8200)
    p.add_argument("--decoder-host", default="127.0.0.1")
    p.add_argument("--connector", default="nixlv2", choices=["nixlv2", "nixl", "sglang", "kvx"])
    p.add_argument("--data-parallel-size", type=int, default=1)
    p.add_argument("--enable-prefiller-sampling", action="store_true")
    p.add_argument("--allowed-prefill-hosts", default="")
    p.add_argument("--secure-proxy", action="store_true")
    p.add_argument("--zap-log-level", default="info")
    a = p.parse_args(argv)
    logging.basicConfig(level=getattr(logging, a.zap_log_level.upper(), logging.INFO))
    conn = "nixlv2" if a.connector in ("nixl", "kvx") else a.connector
    allowed = [x for x in a.allowed_prefill_hosts.split(",") if x]

    async def run():
        runners = []
        for r in range(a.data_parallel_size):
            sc = RoutingSidecar(f"http://{a.decoder_host}:{a.vllm_port + r}", conn, a.enable_prefiller_sampling,
                                allowed, secure_prefill=a.secure_proxy)
            runner = web.AppRunner(sc.app(), access_log=None)
            await runner.setup()
            await web.TCPSite(runner, "0.0.0.0", a.port + r).start()
            runners.append(runner)
        log.info("sidecar on :%d..%d -> decoder :%d..", a.port, a.port + a.data_parallel_size - 1, a.vllm_port)
        while True:
            await asyncio.sleep(3600)

    asyncio.run(run())


if __name__ == "__main__":
    main()
