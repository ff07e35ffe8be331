"""EPP as an Envoy ext_proc v3 server (llmd_amd/router/extproc.py): an Envoy
emulator drives the FULL_DUPLEX_STREAMED protocol of the reference's
envoy.yaml (request headers, body chunks, response headers and streamed body)
over real gRPC and forwards to engine simulators at the destination the EPP
returns (x-gateway-destination-endpoint header + envoy.lb metadata), the way
Envoy's ORIGINAL_DST cluster would. No Envoy binary in this image: the emulator
is the client side of the contract."""
import asyncio
import json

import aiohttp
import grpc
import pytest

from llmd_amd.router import headers as H
from llmd_amd.router.api import ControlPlane
from llmd_amd.router.datalayer import EndpointStore, endpoints_from_yaml
from llmd_amd.router.epp import EPP
from llmd_amd.router.extproc import EXT_PROC_SERVICE, PB, ExtProcServer
from llmd_amd.sim.server import start_sim

CONFIG = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: queue-scorer
- type: prefix-cache-scorer
- type: max-score-picker
schedulingProfiles:
- name: default
  plugins:
  - {pluginRef: queue-scorer, weight: 1}
  - {pluginRef: prefix-cache-scorer, weight: 3}
  - {pluginRef: max-score-picker}
"""


def _hdrs(d, eos):
    m = PB["HttpHeaders"]()
    for k, v in d.items():
        h = m.headers.headers.add()
        h.key = k
        h.raw_value = str(v).encode()
    m.end_of_stream = eos
    return m


class EnvoyEmulator:
    """Client side of ext_proc for one HTTP request, as Envoy's ext_proc filter
    runs it with request/response body mode FULL_DUPLEX_STREAMED."""

    def __init__(self, channel):
        self.call = channel.stream_stream(f"/{EXT_PROC_SERVICE}/Process",
                                          request_serializer=PB["ProcessingRequest"].SerializeToString,
                                          response_deserializer=PB["ProcessingResponse"].FromString)

    async def request(self, session, path, body: bytes, extra_headers=None, chunk=37):
        q: asyncio.Queue = asyncio.Queue()

        async def gen():
            while True:
                m = await q.get()
                if m is None:
                    return
                yield m

        stream = self.call(gen())
        it = stream.__aiter__()
        hdrs = {":method": "POST", ":path": path, ":authority": "gw", "content-type": "application/json",
                "content-length": str(len(body))}
        hdrs.update(extra_headers or {})
        r = PB["ProcessingRequest"]()
        r.request_headers.CopyFrom(_hdrs(hdrs, False))
        await q.put(r)
        for i in range(0, len(body), chunk):  # body in several chunks, the last one ends the stream
            r = PB["ProcessingRequest"]()
            r.request_body.body = body[i:i + chunk]
            r.request_body.end_of_stream = i + chunk >= len(body)
            await q.put(r)
        first = await it.__anext__()
        kind = first.WhichOneof("response")
        if kind == "immediate_response":
            await q.put(None)
            ir = first.immediate_response
            hm = {o.header.key: o.header.raw_value.decode() for o in ir.headers.set_headers}
            return {"immediate": ir.status.code, "body": ir.body, "headers": hm}
        assert kind == "request_headers"
        seth = {o.header.key: o.header.raw_value.decode()
                for o in first.request_headers.response.header_mutation.set_headers}
        meta = dict(first.dynamic_metadata.fields["envoy.lb"].struct_value.fields)
        dest = seth[H.DESTINATION]
        assert meta[H.DESTINATION].string_value == dest
        bodyresp = await it.__anext__()
        sb = bodyresp.request_body.response.body_mutation.streamed_response
        assert sb.end_of_stream
        up_body = sb.body
        assert int(seth["content-length"]) == len(up_body)
        up_headers = {k: v for k, v in seth.items() if k not in ("content-length", H.DESTINATION)}
        up_headers["content-type"] = "application/json"
        # ORIGINAL_DST: forward to the picked endpoint, stream the response through ext_proc
        out = bytearray()
        async with session.post(f"http://{dest}{path}", data=up_body, headers=up_headers) as resp:
            r = PB["ProcessingRequest"]()
            r.response_headers.CopyFrom(_hdrs({":status": resp.status, "content-type": resp.content_type}, False))
            await q.put(r)
            hr = await it.__anext__()
            assert hr.WhichOneof("response") == "response_headers"
            async for c in resp.content.iter_any():
                r = PB["ProcessingRequest"]()
                r.response_body.body = c
                await q.put(r)
                br = await it.__anext__()
                out += br.response_body.response.body_mutation.streamed_response.body
            r = PB["ProcessingRequest"]()
            r.response_body.end_of_stream = True
            await q.put(r)
            br = await it.__anext__()
            assert br.response_body.response.body_mutation.streamed_response.end_of_stream
            status = resp.status
        await q.put(None)
        return {"dest": dest, "status": status, "body": bytes(out), "headers": seth}


def test_extproc_full_duplex_routing_streaming_affinity_and_errors():
    async def main():
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001) for _ in range(3)]
        store = EndpointStore()
        epp = EPP(CONFIG, store, ControlPlane())
        for e in endpoints_from_yaml({"endpoints": [
                {"name": f"s{i}", "address": "127.0.0.1", "port": p} for i, (_, _, p) in enumerate(sims)]}):
            await store.add(e)
        srv = ExtProcServer(epp)
        port = await srv.start(0, host="127.0.0.1")
        async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch, aiohttp.ClientSession() as s:
            health = ch.unary_unary("/grpc.health.v1.Health/Check",
                                    request_serializer=PB["HealthCheckRequest"].SerializeToString,
                                    response_deserializer=PB["HealthCheckResponse"].FromString)
            hr = PB["HealthCheckRequest"]()
            hr.service = EXT_PROC_SERVICE
            assert (await health(hr)).status == 1  # SERVING
            env = EnvoyEmulator(ch)
            prompt = "the quick brown fox " * 40
            body = json.dumps({"model": "m", "prompt": prompt, "max_tokens": 4}).encode()
            r1 = await env.request(s, "/v1/completions", body)
            assert r1["status"] == 200 and json.loads(r1["body"])["usage"]["completion_tokens"] == 4
            # same long prompt again: the prefix-cache scorer keeps it on the same endpoint
            r2 = await env.request(s, "/v1/completions", body)
            assert r2["dest"] == r1["dest"]
            # streamed response passes through ext_proc chunk by chunk, unchanged
            sb = json.dumps({"model": "m", "prompt": "hello", "max_tokens": 5, "stream": True,
                             "stream_options": {"include_usage": True}}).encode()
            r3 = await env.request(s, "/v1/completions", sb, {"x-request-id": "rid-7"})
            assert r3["status"] == 200 and r3["body"].strip().endswith(b"[DONE]")
            assert r3["headers"][H.REQUEST_ID] == "rid-7"
            # every request completed: in-flight accounting back to zero
            assert sum(epp.ctx.inflight_requests.values()) == 0
            # malformed body -> ImmediateResponse from the EPP (parser 400)
            bad = await env.request(s, "/v1/completions", b"{not json")
            assert bad["immediate"] == 400
            # empty pool -> 503 ImmediateResponse, health NOT_SERVING
            for e in list(store.all()):
                await store.remove(e.key)
            r4 = await env.request(s, "/v1/completions", body)
            assert r4["immediate"] == 503
            assert (await health(hr)).status == 2
        text = epp.render_metrics().decode()
        assert "inference_objective_request_total" in text or "llm_d" in text
        await srv.stop()
        for sm in sims:
            await sm[0].cleanup()

    asyncio.run(main())


@pytest.mark.parametrize("mode", ["FailClose"])
def test_extproc_standby_replica_answers_503(mode, tmp_path):
    class Standby:
        is_leader = False

        def start(self):
            pass

        def stop(self):
            pass

    async def main():
        store = EndpointStore()
        epp = EPP(CONFIG, store, ControlPlane())
        srv = ExtProcServer(epp, mode, elector=Standby())
        port = await srv.start(0, host="127.0.0.1")
        async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch, aiohttp.ClientSession() as s:
            r = await EnvoyEmulator(ch).request(s, "/v1/completions", b'{"model": "m", "prompt": "x"}')
            assert r["immediate"] == 503
        await srv.stop()

    asyncio.run(main())
