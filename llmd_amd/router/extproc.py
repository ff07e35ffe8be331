"""Envoy External Processing (ext_proc v3) server for the EPP (SURVEY C08/C07,
M14): the reference's standalone and Gateway deployments put Envoy (or
kgateway / Istio / GKE) in front and call the Endpoint Picker over gRPC on
:9002 with ``request_body_mode`` / ``response_body_mode`` ``FULL_DUPLEX_STREAMED``
(guides/no-kubernetes-deployment/router/envoy/envoy.yaml:56-72,
docs/architecture/core/router/epp/README.md:11-16). This module serves that
contract with the same in-process ``EPP`` the aiohttp proxy uses, so an
existing Envoy config can point at it unchanged.

Per stream (one HTTP request):
  request_headers  -> remembered (a body-less request is routed at once)
  request_body*    -> buffered; at end_of_stream the EPP schedules it, then
                      HeadersResponse (x-gateway-destination-endpoint + the
                      decision's headers, content-length of the possibly
                      rewritten body; the same destination in dynamic metadata
                      ``envoy.lb``) and the body as one StreamedBodyResponse
  response_headers -> status to the response processors, CONTINUE
  response_body*   -> each chunk to the response processors and streamed back
                      unchanged; at end_of_stream usage/TTFT/TPOT complete the
                      request (in-flight accounting, latency samples)
  trailers         -> CONTINUE
Scheduling errors become an ImmediateResponse with the EPP's status and
``x-llm-d-request-dropped-reason``.

gRPC health (grpc.health.v1.Health/Check) answers SERVING on the ext_proc
port (Envoy health-checks the ext_proc cluster there, envoy.yaml:113-120)
and on ``--grpc-health-port``.

No protoc in this image: the message descriptors are built in code from the
public envoy / grpc-health field numbers (only the fields this server reads or
writes; unknown fields are skipped by the protobuf parser).

CLI (EPP flags, guides/no-kubernetes-deployment/README.md:153-190):
  python -m llmd_amd.router.extproc --config-file epp.yaml --endpoints-file endpoints.yaml \\
      --grpc-port 9002 --grpc-health-port 9003 --metrics-port 9090 --pool-name pool
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import random
import time
from typing import Optional

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, struct_pb2

from . import headers as H
from .epp import EPP, Decision
from .proxy import INFERENCE_PATHS, _find_usage
from ..utils.tracing import span
from .types import CIHeaders, InferenceRequest, SchedulingError

log = logging.getLogger("llmd.router.extproc")

EXT_PROC_SERVICE = "envoy.service.ext_proc.v3.ExternalProcessor"
HEALTH_SERVICE = "grpc.health.v1.Health"

# --------------------------------------------------------------------- protos
_F = descriptor_pb2.FieldDescriptorProto
_T = {"string": _F.TYPE_STRING, "bytes": _F.TYPE_BYTES, "bool": _F.TYPE_BOOL, "int32": _F.TYPE_INT32,
      "uint32": _F.TYPE_UINT32, "enum": _F.TYPE_ENUM, "msg": _F.TYPE_MESSAGE}


def _msg(fdp, name, fields, oneofs=(), enums=()):
    m = fdp.message_type.add(name=name)
    for en, vals in enums:
        e = m.enum_type.add(name=en)
        for vn, vv in vals:
            e.value.add(name=vn, number=vv)
    for o in oneofs:
        m.oneof_decl.add(name=o)
    for f in fields:
        fname, num, typ = f[0], f[1], f[2]
        tname = f[3] if len(f) > 3 else None
        rep = f[4] if len(f) > 4 else False
        oneof = f[5] if len(f) > 5 else None
        fd = m.field.add(name=fname, number=num, type=_T[typ],
                         label=_F.LABEL_REPEATED if rep else _F.LABEL_OPTIONAL)
        if tname:
            fd.type_name = tname
        if oneof is not None:
            fd.oneof_index = oneofs.index(oneof)
    return m


def _build_pool():
    pool = descriptor_pool.DescriptorPool()
    sfd = descriptor_pb2.FileDescriptorProto()
    struct_pb2.DESCRIPTOR.CopyToProto(sfd)
    pool.Add(sfd)

    base = descriptor_pb2.FileDescriptorProto(name="envoy/config/core/v3/base.proto",
                                              package="envoy.config.core.v3", syntax="proto3")
    _msg(base, "HeaderValue", [("key", 1, "string"), ("value", 2, "string"), ("raw_value", 3, "bytes")])
    _msg(base, "HeaderValueOption",
         [("header", 1, "msg", ".envoy.config.core.v3.HeaderValue"),
          ("append_action", 3, "enum", ".envoy.config.core.v3.HeaderValueOption.HeaderAppendAction"),
          ("keep_empty_value", 4, "bool")],
         enums=[("HeaderAppendAction", [("APPEND_IF_EXISTS_OR_ADD", 0), ("ADD_IF_ABSENT", 1),
                                        ("OVERWRITE_IF_EXISTS_OR_ADD", 2), ("OVERWRITE_IF_EXISTS", 3)])])
    _msg(base, "HeaderMap", [("headers", 1, "msg", ".envoy.config.core.v3.HeaderValue", True)])
    pool.Add(base)

    st = descriptor_pb2.FileDescriptorProto(name="envoy/type/v3/http_status.proto", package="envoy.type.v3",
                                            syntax="proto3")
    _msg(st, "HttpStatus", [("code", 1, "uint32")])  # StatusCode enum on the wire: a varint
    pool.Add(st)

    ep = descriptor_pb2.FileDescriptorProto(
        name="envoy/service/ext_proc/v3/external_processor.proto", package="envoy.service.ext_proc.v3",
        syntax="proto3", dependency=["envoy/config/core/v3/base.proto", "envoy/type/v3/http_status.proto",
                                     "google/protobuf/struct.proto"])
    P = ".envoy.service.ext_proc.v3."
    C = ".envoy.config.core.v3."
    _msg(ep, "HttpHeaders", [("headers", 1, "msg", C + "HeaderMap"), ("end_of_stream", 3, "bool")])
    _msg(ep, "HttpBody", [("body", 1, "bytes"), ("end_of_stream", 2, "bool")])
    _msg(ep, "HttpTrailers", [("trailers", 1, "msg", C + "HeaderMap")])
    _msg(ep, "ProcessingRequest",
         [("request_headers", 2, "msg", P + "HttpHeaders", False, "request"),
          ("response_headers", 3, "msg", P + "HttpHeaders", False, "request"),
          ("request_body", 4, "msg", P + "HttpBody", False, "request"),
          ("response_body", 5, "msg", P + "HttpBody", False, "request"),
          ("request_trailers", 6, "msg", P + "HttpTrailers", False, "request"),
          ("response_trailers", 7, "msg", P + "HttpTrailers", False, "request"),
          ("observability_mode", 10, "bool")], oneofs=("request",))
    _msg(ep, "HeaderMutation", [("set_headers", 1, "msg", C + "HeaderValueOption", True),
                                ("remove_headers", 2, "string", None, True)])
    _msg(ep, "StreamedBodyResponse", [("body", 1, "bytes"), ("end_of_stream", 2, "bool")])
    _msg(ep, "BodyMutation", [("body", 1, "bytes", None, False, "mutation"),
                              ("clear_body", 2, "bool", None, False, "mutation"),
                              ("streamed_response", 3, "msg", P + "StreamedBodyResponse", False, "mutation")],
         oneofs=("mutation",))
    _msg(ep, "CommonResponse",
         [("status", 1, "enum", P + "CommonResponse.ResponseStatus"),
          ("header_mutation", 2, "msg", P + "HeaderMutation"), ("body_mutation", 3, "msg", P + "BodyMutation"),
          ("trailers", 4, "msg", C + "HeaderMap"), ("clear_route_cache", 5, "bool")],
         enums=[("ResponseStatus", [("CONTINUE", 0), ("CONTINUE_AND_REPLACE", 1)])])
    _msg(ep, "HeadersResponse", [("response", 1, "msg", P + "CommonResponse")])
    _msg(ep, "BodyResponse", [("response", 1, "msg", P + "CommonResponse")])
    _msg(ep, "TrailersResponse", [("header_mutation", 1, "msg", P + "HeaderMutation")])
    _msg(ep, "ImmediateResponse", [("status", 1, "msg", ".envoy.type.v3.HttpStatus"),
                                   ("headers", 2, "msg", P + "HeaderMutation"), ("body", 3, "bytes"),
                                   ("details", 5, "string")])
    _msg(ep, "ProcessingResponse",
         [("request_headers", 1, "msg", P + "HeadersResponse", False, "response"),
          ("response_headers", 2, "msg", P + "HeadersResponse", False, "response"),
          ("request_body", 3, "msg", P + "BodyResponse", False, "response"),
          ("response_body", 4, "msg", P + "BodyResponse", False, "response"),
          ("request_trailers", 5, "msg", P + "TrailersResponse", False, "response"),
          ("response_trailers", 6, "msg", P + "TrailersResponse", False, "response"),
          ("immediate_response", 7, "msg", P + "ImmediateResponse", False, "response"),
          ("dynamic_metadata", 8, "msg", ".google.protobuf.Struct")], oneofs=("response",))
    pool.Add(ep)

    hp = descriptor_pb2.FileDescriptorProto(name="grpc/health/v1/health.proto", package="grpc.health.v1",
                                            syntax="proto3")
    _msg(hp, "HealthCheckRequest", [("service", 1, "string")])
    _msg(hp, "HealthCheckResponse", [("status", 1, "enum", ".grpc.health.v1.HealthCheckResponse.ServingStatus")],
         enums=[("ServingStatus", [("UNKNOWN", 0), ("SERVING", 1), ("NOT_SERVING", 2), ("SERVICE_UNKNOWN", 3)])])
    pool.Add(hp)

    def cls(n):
        return message_factory.GetMessageClass(pool.FindMessageTypeByName(n))

    names = ["envoy.config.core.v3.HeaderValue", "envoy.config.core.v3.HeaderValueOption",
             "envoy.config.core.v3.HeaderMap", "envoy.type.v3.HttpStatus"] + \
            [f"envoy.service.ext_proc.v3.{n}" for n in (
                "HttpHeaders", "HttpBody", "HttpTrailers", "ProcessingRequest", "HeaderMutation",
                "StreamedBodyResponse", "BodyMutation", "CommonResponse", "HeadersResponse", "BodyResponse",
                "TrailersResponse", "ImmediateResponse", "ProcessingResponse")] + \
            ["grpc.health.v1.HealthCheckRequest", "grpc.health.v1.HealthCheckResponse"]
    return {n.rsplit(".", 1)[1]: cls(n) for n in names}


PB = _build_pool()


def _hdr_value(h) -> str:
    return h.value if h.value else h.raw_value.decode("utf-8", errors="replace")


def header_mutation(hdrs: dict, remove=()):
    m = PB["HeaderMutation"]()
    for k, v in hdrs.items():
        o = m.set_headers.add()
        o.header.key = k.lower()
        o.header.raw_value = str(v).encode()
        o.append_action = 2  # OVERWRITE_IF_EXISTS_OR_ADD
    m.remove_headers.extend(remove)
    return m


def _metadata(dest: str):
    s = struct_pb2.Struct()
    s.update({"envoy.lb": {H.DESTINATION: dest}})
    return s


class _Stream:
    """State of one ext_proc stream (one proxied HTTP request)."""

    def __init__(self, srv: "ExtProcServer"):
        self.srv = srv
        self.headers: dict = {}
        self.body = bytearray()
        self.d: Optional[Decision] = None
        self.t0 = 0.0
        self.first: Optional[float] = None
        self.last: Optional[float] = None
        self.tail = b""
        self.status: Optional[int] = None
        self.done = False

    def _routing(self, d: Decision, payload: Optional[bytes]):
        R = PB["ProcessingResponse"]()
        cr = R.request_headers.response
        hdrs = dict(d.headers)
        if payload is not None:
            hdrs["content-length"] = str(len(payload))
        hdrs[H.REQUEST_ID] = d.req.request_id
        cr.header_mutation.CopyFrom(header_mutation(hdrs))
        cr.clear_route_cache = True
        R.dynamic_metadata.ParseFromString(_metadata(d.endpoint.key).SerializeToString())
        return R

    def _body_out(self, payload: bytes, response: bool):
        R = PB["ProcessingResponse"]()
        br = R.response_body if response else R.request_body
        sb = br.response.body_mutation.streamed_response
        sb.body = payload
        sb.end_of_stream = True
        return R

    def _immediate(self, status: int, msg: str, reason: str = ""):
        R = PB["ProcessingResponse"]()
        ir = R.immediate_response
        ir.status.code = status
        hdrs = {"content-type": "application/json"}
        if reason:
            hdrs[H.DROPPED_REASON] = reason
        ir.headers.CopyFrom(header_mutation(hdrs))
        ir.body = json.dumps({"error": {"message": msg, "code": status}}).encode()
        ir.details = msg
        return R

    def _random_route(self):
        eps = self.srv.epp.store.all()
        if not eps:
            return None
        ep = random.choice(eps)
        return Decision(InferenceRequest(self.headers.get(":path", "/"), {}, CIHeaders(self.headers), 0), ep,
                        {H.DESTINATION: ep.key})

    async def on_request_headers(self, msg):
        self.t0 = time.monotonic()
        self.headers = {h.key.lower(): _hdr_value(h) for h in msg.headers.headers}
        if msg.end_of_stream:  # no body (GET /v1/models, health): route to any endpoint
            d = self._random_route()
            if d is None:
                return [self._immediate(503, "no ready endpoints in the pool")]
            self.done = True  # nothing to account for
            return [self._routing(d, None)]
        return []

    async def on_request_body(self, msg):
        self.body += msg.body
        if not msg.end_of_stream:
            return []  # FULL_DUPLEX_STREAMED: answer once the whole body is here
        body = bytes(self.body)
        path = self.headers.get(":path", "/").split("?")[0]
        if self.headers.get(":method", "POST") != "POST" or path not in INFERENCE_PATHS:
            d = self._random_route()
            if d is None:
                return [self._immediate(503, "no ready endpoints in the pool")]
            self.done = True
            return [self._routing(d, body), self._body_out(body, False)]
        with span("gateway.request", {"path": path}, traceparent=self.headers.get("traceparent")):
            try:
                d = await self.srv.epp.handle(path, body, dict(self.headers))
            except SchedulingError as e:
                self.done = True
                return [self._immediate(e.status, str(e), e.reason or "")]
            except Exception as e:  # noqa: BLE001 - EPP failure: FailOpen / FailClose
                log.exception("EPP failure")
                d = self._random_route() if self.srv.failure_mode == "FailOpen" else None
                if d is None:
                    self.done = True
                    return [self._immediate(503, f"endpoint picker failed: {e}")]
                self.done = True  # fail-open requests are not accounted
        self.d = d
        payload = d.body if d.body is not None else body
        return [self._routing(d, payload), self._body_out(payload, False)]

    def on_response_headers(self, msg):
        hdrs = {h.key.lower(): _hdr_value(h) for h in msg.headers.headers}
        try:
            self.status = int(hdrs.get(":status", "200"))
        except ValueError:
            self.status = None
        if self.d is not None and not self.done:
            self.srv.epp.on_response_headers(self.d, self.status or 0,
                                             {k: v for k, v in hdrs.items() if not k.startswith(":")})
        R = PB["ProcessingResponse"]()
        R.response_headers.response.status = 0
        if msg.end_of_stream:
            self.complete()
        return [R]

    def on_response_body(self, msg):
        now = time.monotonic()
        chunk = bytes(msg.body)
        if chunk:
            if self.first is None:
                self.first = now
            self.last = now
            if self.d is not None and self.d.req.data.get("grpc"):
                # gRPC frames must stay whole for the usage parse (bounded)
                self.tail = (self.tail + chunk) if len(self.tail) < (8 << 20) else self.tail
            else:
                self.tail = (self.tail + chunk)[-65536:]
            if self.d is not None and not self.done:
                self.srv.epp.on_response_chunk(self.d, chunk, now)
        R = PB["ProcessingResponse"]()
        sb = R.response_body.response.body_mutation.streamed_response
        sb.body = chunk
        sb.end_of_stream = msg.end_of_stream
        if msg.end_of_stream:
            self.complete()
        return [R]

    def complete(self, aborted: bool = False):
        if self.done or self.d is None:
            self.done = True
            return
        self.done = True
        end = time.monotonic()
        info = {"status": None if aborted else self.status, "duration": end - self.t0, "ttft": None,
                "usage": _find_usage(self.tail, grpc=bool(self.d.req.data.get("grpc")))}
        if self.first is not None and (self.d.req.stream or self.status == 200):
            info["ttft"] = self.first - self.t0
        n = (info["usage"] or {}).get("completion_tokens") or 0
        if self.first is not None and n > 1 and self.last is not None:
            info["tpot"] = (self.last - self.first) / (n - 1)
        self.srv.epp.on_response_complete(self.d, info)


class ExtProcServer:
    def __init__(self, epp: EPP, failure_mode: str = "FailOpen", elector=None):
        self.epp = epp
        self.failure_mode = failure_mode
        self.elector = elector
        self.servers: list = []

    @property
    def active(self) -> bool:
        return self.elector is None or self.elector.is_leader

    async def process(self, request_iterator, context):
        st = _Stream(self)
        try:
            async for msg in request_iterator:
                kind = msg.WhichOneof("request")
                if not self.active:
                    yield st._immediate(503, "endpoint picker standby (not the HA leader)")
                    return
                if kind == "request_headers":
                    outs = await st.on_request_headers(msg.request_headers)
                elif kind == "request_body":
                    outs = await st.on_request_body(msg.request_body)
                elif kind == "request_trailers":
                    R = PB["ProcessingResponse"]()
                    R.request_trailers.SetInParent()
                    outs = [R]
                elif kind == "response_headers":
                    outs = st.on_response_headers(msg.response_headers)
                elif kind == "response_body":
                    outs = st.on_response_body(msg.response_body)
                elif kind == "response_trailers":
                    R = PB["ProcessingResponse"]()
                    R.response_trailers.SetInParent()
                    st.complete()
                    outs = [R]
                else:
                    outs = []
                for o in outs:
                    yield o
        finally:
            st.complete(aborted=True)  # client went away mid-stream: release in-flight accounting

    async def health_check(self, req, context):
        R = PB["HealthCheckResponse"]()
        ok = self.active and bool(self.epp.store.all())
        if req.service not in ("", EXT_PROC_SERVICE):
            R.status = 3  # SERVICE_UNKNOWN
        else:
            R.status = 1 if ok else 2
        return R

    def handlers(self):
        ext = grpc.method_handlers_generic_handler(EXT_PROC_SERVICE, {
            "Process": grpc.stream_stream_rpc_method_handler(
                self.process, request_deserializer=PB["ProcessingRequest"].FromString,
                response_serializer=PB["ProcessingResponse"].SerializeToString)})
        health = grpc.method_handlers_generic_handler(HEALTH_SERVICE, {
            "Check": grpc.unary_unary_rpc_method_handler(
                self.health_check, request_deserializer=PB["HealthCheckRequest"].FromString,
                response_serializer=PB["HealthCheckResponse"].SerializeToString)})
        return ext, health

    async def start(self, port: int, health_port: Optional[int] = None, host: str = "0.0.0.0") -> int:
        await self.epp.start()
        if self.elector is not None:
            self.elector.start()
        ext, health = self.handlers()
        s = grpc.aio.server(options=[("grpc.max_receive_message_length", 256 << 20),
                                     ("grpc.max_send_message_length", 256 << 20)])
        s.add_generic_rpc_handlers((ext, health))
        bound = s.add_insecure_port(f"{host}:{port}")
        await s.start()
        self.servers.append(s)
        if health_port:
            hs = grpc.aio.server()
            hs.add_generic_rpc_handlers((health,))
            hs.add_insecure_port(f"{host}:{health_port}")
            await hs.start()
            self.servers.append(hs)
        log.info("ext_proc EPP on :%d (health :%s)", bound, health_port)
        return bound

    async def stop(self):
        for s in self.servers:
            await s.stop(grace=1.0)
        self.servers = []
        if self.elector is not None:
            self.elector.stop()
        await self.epp.stop()


def main(argv=None):
    from aiohttp import web

    from .api import ControlPlane
    from .datalayer import EndpointStore, FileDiscovery, endpoints_from_yaml
    from .proxy import DEFAULT_CONFIG

    p = argparse.ArgumentParser("llmd-amd EPP (Envoy ext_proc server)")
    p.add_argument("--config-file")
    p.add_argument("--config-text")
    p.add_argument("--endpoints-file", help="file-discovery endpoints.yaml")
    p.add_argument("--endpoints", default="", help="comma list ip:port[:role]")
    p.add_argument("--control-plane", help="YAML with InferencePool/Objective/ModelRewrite docs")
    p.add_argument("--pool-name", default="pool")
    p.add_argument("--pool-namespace", default="default")
    p.add_argument("--grpc-port", type=int, default=9002)
    p.add_argument("--grpc-health-port", type=int, default=9003)
    p.add_argument("--metrics-port", type=int, default=9090)
    p.add_argument("--failure-mode", default="FailOpen", choices=["FailOpen", "FailClose"])
    p.add_argument("--ha-enable-leader-election", action="store_true")
    p.add_argument("--ha-lease-file", default=None)
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

        elector = LeaseElector(a.ha_lease_file or f"/tmp/llmd-epp-{a.pool_namespace}-{a.pool_name}.lease")
    srv = ExtProcServer(epp, a.failure_mode, elector)

    async def run():
        if a.endpoints_file:
            fd = FileDiscovery("file-discovery", {"path": a.endpoints_file, "watchFile": True})
            await fd.start_watch(store)
        if a.endpoints:
            eps = []
            for i, item in enumerate(x for x in a.endpoints.split(",") if x):
                parts = item.split(":")
                labels = {"llm-d.ai/role": parts[2]} if len(parts) > 2 else {}
                eps.append({"name": f"ep{i}", "address": parts[0], "port": int(parts[1]), "labels": labels})
            for e in endpoints_from_yaml({"endpoints": eps}):
                await store.add(e)
        await srv.start(a.grpc_port, a.grpc_health_port)
        mapp = web.Application()

        async def metrics(_):
            return web.Response(body=epp.render_metrics(), content_type="text/plain")
        mapp.router.add_get("/metrics", metrics)
        mr = web.AppRunner(mapp)
        await mr.setup()
        await web.TCPSite(mr, "0.0.0.0", a.metrics_port).start()
        while True:
            await asyncio.sleep(3600)

    asyncio.run(run())


if __name__ == "__main__":
    main()
