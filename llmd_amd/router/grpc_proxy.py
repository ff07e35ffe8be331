"""gRPC (h2c) data plane of the standalone router: the vLLM gRPC engine API
(``vllm.grpc.engine.VllmEngine/Generate`` and ``/Embed``) through the
in-process EPP - the gRPC counterpart of router/proxy.py (aiohttp speaks
HTTP/1.1 only). In the reference this traffic crosses the gateway as HTTP/2
cleartext and the EPP decodes the frames to route
(docs/api-reference/epp-grpc-apis.md:1-57; InferencePool ``appProtocol:
kubernetes.io/h2c``).

Per call: the request message (raw bytes) is framed and handed to the EPP
(``vllmgrpc-parser`` -> flow control -> producers -> scheduler), gRPC metadata
play the HTTP headers (x-llm-d-inference-objective, fairness id, SLOs,
x-request-id), the call is forwarded unchanged to the picked endpoint's gRPC
port with the decision headers added as metadata, the response stream is
relayed back message by message and its usage (``complete`` counts, or the
counted ``chunk`` tokens), TTFT and TPOT complete the request in the EPP.
EPP rejections map to gRPC status codes (429 -> RESOURCE_EXHAUSTED, 503 ->
UNAVAILABLE, 400 -> INVALID_ARGUMENT) with the dropped-reason in the trailing
metadata.

Endpoint ports: the pool's endpoints are the engines' HTTP ports (metrics are
scraped there); ``grpc_target`` maps one to its gRPC port - an explicit map,
or a fixed offset (``--grpc-upstream-port-offset``).
"""
from __future__ import annotations

import logging
import time
from typing import Callable, Optional

import grpc

from llmd_amd.serving import vllm_grpc as vg

from . import headers as H
from .epp import EPP
from .types import SchedulingError

log = logging.getLogger("llmd.router.grpc")

_STATUS = {400: grpc.StatusCode.INVALID_ARGUMENT, 429: grpc.StatusCode.RESOURCE_EXHAUSTED,
           503: grpc.StatusCode.UNAVAILABLE, 500: grpc.StatusCode.INTERNAL}
_RESERVED = {"content-type", "te", "user-agent", "grpc-accept-encoding", "grpc-encoding", "grpc-timeout"}


def _identity(x):
    return x


class GrpcRouter:
    def __init__(self, epp: EPP, grpc_target: Callable[[str], str]):
        self.epp = epp
        self.grpc_target = grpc_target
        self.channels: dict[str, grpc.aio.Channel] = {}
        self.server: Optional[grpc.aio.Server] = None

    def _channel(self, target: str) -> grpc.aio.Channel:
        ch = self.channels.get(target)
        if ch is None:
            ch = self.channels[target] = grpc.aio.insecure_channel(
                target, options=[("grpc.max_receive_message_length", 64 << 20),
                                 ("grpc.max_send_message_length", 64 << 20)])
        return ch

    async def _decide(self, path: str, raw: bytes, context):
        md = {k.lower(): v for k, v in (context.invocation_metadata() or ()) if isinstance(v, str)}
        try:
            return await self.epp.handle(path, vg.frame(raw), md), md
        except SchedulingError as e:
            if e.reason:
                context.set_trailing_metadata(((H.DROPPED_REASON.lower(), e.reason),))
            await context.abort(_STATUS.get(e.status, grpc.StatusCode.UNKNOWN), str(e))

    def _upstream_md(self, md: dict, d) -> tuple:
        out = {k: v for k, v in md.items() if k not in _RESERVED and not k.startswith(":")}
        out.update({k.lower(): str(v) for k, v in d.headers.items()})
        out[H.REQUEST_ID.lower()] = d.req.request_id
        return tuple(out.items())

    async def generate(self, raw: bytes, context):
        d, md = await self._decide(vg.GENERATE, raw, context)
        target = self.grpc_target(d.endpoint.key)
        call = self._channel(target).unary_stream(vg.GENERATE, request_serializer=_identity,
                                                  response_deserializer=_identity)
        t0 = time.monotonic()
        info = {"ttft": None, "usage": None, "status": None}
        first = last = None
        msgs = []
        self.epp.on_response_headers(d, 200, {"content-type": "application/grpc"})
        try:
            async for m in call(raw, metadata=self._upstream_md(md, d)):
                now = time.monotonic()
                first = first or now
                last = now
                msgs.append(m)
                self.epp.on_response_chunk(d, vg.frame(m), now)
                yield m
            info["status"] = 200
        except grpc.aio.AioRpcError as e:
            info["status"] = 502
            await context.abort(e.code(), f"upstream {target}: {e.details()}")
        finally:
            info["duration"] = time.monotonic() - t0
            info["usage"] = vg.usage_of_responses(msgs) if msgs else None
            if first is not None:
                info["ttft"] = first - t0
            n = (info["usage"] or {}).get("completion_tokens") or 0
            if first is not None and n > 1 and last is not None and len(msgs) > 1:
                info["tpot"] = (last - first) / (n - 1)
            self.epp.on_response_complete(d, info)

    async def embed(self, raw: bytes, context):
        d, md = await self._decide(vg.EMBED, raw, context)
        target = self.grpc_target(d.endpoint.key)
        call = self._channel(target).unary_unary(vg.EMBED, request_serializer=_identity,
                                                 response_deserializer=_identity)
        t0 = time.monotonic()
        info = {"ttft": None, "usage": None, "status": 200}
        try:
            out = await call(raw, metadata=self._upstream_md(md, d))
            r = vg.PB["EmbedResponse"].FromString(out)
            info["usage"] = {"prompt_tokens": r.prompt_tokens, "completion_tokens": 0,
                             "total_tokens": r.prompt_tokens}
            return out
        except grpc.aio.AioRpcError as e:
            info["status"] = 502
            await context.abort(e.code(), f"upstream {target}: {e.details()}")
        finally:
            info["duration"] = time.monotonic() - t0
            self.epp.on_response_complete(d, info)

    def handler(self):
        return grpc.method_handlers_generic_handler(vg.SERVICE, {
            "Generate": grpc.unary_stream_rpc_method_handler(self.generate, request_deserializer=_identity,
                                                             response_serializer=_identity),
            "Embed": grpc.unary_unary_rpc_method_handler(self.embed, request_deserializer=_identity,
                                                         response_serializer=_identity)})

    async def start(self, port: int, host: str = "0.0.0.0") -> int:
        s = grpc.aio.server(options=[("grpc.max_receive_message_length", 64 << 20),
                                     ("grpc.max_send_message_length", 64 << 20)])
        s.add_generic_rpc_handlers((self.handler(),))
        bound = s.add_insecure_port(f"{host}:{port}")
        await s.start()
        self.server = s
        log.info("gRPC (h2c) router data plane on :%d", bound)
        return bound

    async def stop(self):
        if self.server is not None:
            await self.server.stop(grace=1.0)
        for ch in self.channels.values():
            await ch.close()
        self.channels.clear()


def offset_target(offset: int, overrides: Optional[dict] = None) -> Callable[[str], str]:
    """endpoint key host:port -> host:(port + offset), unless listed in overrides."""
    overrides = dict(overrides or {})

    def f(key: str) -> str:
        if key in overrides:
            return overrides[key]
        host, port = key.rsplit(":", 1)
        return f"{host}:{int(port) + offset}"
    return f
