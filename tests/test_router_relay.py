"""Native router data plane (csrc/relay/relay.cpp via router/relay.py): one
llmd-relay process relays requests and streamed responses for an EPP that
serves decisions over its Unix socket (router/workers.py EppServer).

Checked against router/proxy.py's contract:
* health / passthrough / metrics on the data-plane port;
* the upstream sees the client's headers minus hop-by-hop ones, the
  decision's headers, ``x-request-id`` and a ``traceparent`` continuing the
  client's trace;
* JSON and SSE (chunked) responses arrive byte-exact; the EPP's response hooks
  get status, TTFT, TPOT and the usage block parsed from the stream tail;
* prefix affinity across the relay's threads (one EPP);
* EPP rejections keep status + dropped-reason header; a dead endpoint is a 502;
  with the EPP gone, FailClose answers 503;
* chunked request bodies and ``Expect: 100-continue``;
* a client that disconnects mid-stream has its decision completed.
"""
import asyncio
import json
import socket
import time

import aiohttp
import pytest
from aiohttp import web

from llmd_amd.router.api import ControlPlane
from llmd_amd.router.datalayer import EndpointStore, endpoints_from_yaml
from llmd_amd.router.epp import EPP
from llmd_amd.router.relay import relay_binary, spawn
from llmd_amd.router.workers import EppServer
from llmd_amd.sim.server import start_sim
from tests.test_router_e2e import BASE

pytestmark = pytest.mark.skipif(relay_binary() is None, reason="llmd-relay not buildable (no g++)")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _echo_engine():
    """An engine stand-in that reports what it received: JSON echo, an SSE stream, a slow stream."""
    seen = []

    async def completions(req: web.Request):
        body = await req.json()
        seen.append({"headers": dict(req.headers), "body": body})
        n = int(body.get("max_tokens", 3))
        usage = {"prompt_tokens": 7, "completion_tokens": n, "total_tokens": 7 + n}
        if not body.get("stream"):
            return web.json_response({"echo": body, "usage": usage, "headers": dict(req.headers)})
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream", "x-engine": "echo"})
        await resp.prepare(req)
        for i in range(n):
            await resp.write(f"data: {json.dumps({'choices': [{'text': f't{i}'}]})}\n\n".encode())
            await asyncio.sleep(body.get("delay", 0.002))
        await resp.write(f"data: {json.dumps({'choices': [], 'usage': usage})}\n\n".encode())
        await resp.write(b"data: [DONE]\n\n")
        await resp.write_eof()
        return resp

    async def models(req):
        return web.json_response({"data": [{"id": "m"}]})

    app = web.Application()
    app.router.add_post("/v1/completions", completions)
    app.router.add_get("/v1/models", models)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    port = _free_port()
    await web.TCPSite(runner, "127.0.0.1", port).start()
    return runner, port, seen


async def _up(port, relay):
    async with aiohttp.ClientSession() as s:
        for _ in range(200):
            assert relay.poll() is None, "relay exited"
            try:
                async with s.get(f"http://127.0.0.1:{port}/health") as r:
                    if r.status == 200:
                        return
            except aiohttp.ClientError:
                pass
            await asyncio.sleep(0.05)
    raise AssertionError("relay never became healthy")


async def _raw(port, data: bytes, read_until=b"0\r\n\r\n", timeout=5.0):
    r, w = await asyncio.open_connection("127.0.0.1", port)
    w.write(data)
    await w.drain()
    buf = b""
    t = time.monotonic()
    while time.monotonic() - t < timeout:
        try:
            chunk = await asyncio.wait_for(r.read(65536), 0.5)
        except asyncio.TimeoutError:
            continue
        if not chunk:
            break
        buf += chunk
        if read_until in buf or (b"Content-Length:" in buf and _complete(buf)):
            break
    w.close()
    return buf


def _complete(buf: bytes) -> bool:
    head, _, body = buf.partition(b"\r\n\r\n")
    for line in head.split(b"\r\n"):
        if line.lower().startswith(b"content-length:"):
            return len(body) >= int(line.split(b":")[1])
    return False


def test_native_relay_contract(tmp_path):
    async def main():
        engine, eport, seen = await _echo_engine()
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.0005) for _ in range(3)]
        store = EndpointStore()
        epp = EPP(BASE, store, ControlPlane())
        eps = [{"name": "echo", "address": "127.0.0.1", "port": eport}]
        await store.add(endpoints_from_yaml({"endpoints": eps})[0])
        await epp.start()
        infos = []
        orig = epp.on_response_complete

        def record(d, info):
            infos.append(dict(info))
            return orig(d, info)
        epp.on_response_complete = record
        uds = str(tmp_path / "epp.sock")
        srv = EppServer(epp)
        await srv.start(uds)
        port = _free_port()
        relay = spawn(uds, "127.0.0.1", port, 3, "FailClose")
        try:
            await _up(port, relay)
            url = f"http://127.0.0.1:{port}"
            async with aiohttp.ClientSession() as s:
                # JSON: headers forwarded, hop-by-hop dropped, request id + trace continued
                tp = "00-" + "ab" * 16 + "-" + "cd" * 8 + "-01"
                async with s.post(f"{url}/v1/completions?x=1", json={"model": "m", "prompt": "hello", "max_tokens": 3},
                                  headers={"x-custom": "v", "traceparent": tp}) as r:
                    assert r.status == 200
                    out = await r.json()
                h = {k.lower(): v for k, v in out["headers"].items()}
                assert h["x-custom"] == "v" and h["host"] == f"127.0.0.1:{eport}"
                assert h["x-request-id"]
                assert h["traceparent"].startswith("00-" + "ab" * 16 + "-") and h["traceparent"].endswith("-01")
                assert h["traceparent"] != tp
                assert out["echo"]["prompt"] == "hello"
                # SSE through chunked framing, byte-exact, usage reported to the EPP
                async with s.post(f"{url}/v1/completions", json={"model": "m", "prompt": "x", "max_tokens": 5,
                                                                  "stream": True}) as r:
                    assert r.status == 200 and r.headers["x-engine"] == "echo"
                    body = await r.read()
                assert body.count(b"data: ") == 7 and body.endswith(b"data: [DONE]\n\n")
                await asyncio.sleep(0.1)
                last = infos[-1]
                assert last["status"] == 200 and last["usage"]["completion_tokens"] == 5
                assert last["ttft"] is not None and last["ttft"] >= 0 and last["tpot"] > 0
                assert infos[-2]["usage"]["completion_tokens"] == 3
                # passthrough (non-inference path) and /metrics on the data-plane port
                async with s.get(f"{url}/v1/models") as r:
                    assert r.status == 200 and (await r.json())["data"][0]["id"] == "m"
                async with s.get(f"{url}/metrics") as r:
                    assert r.status == 200
                # an EPP rejection keeps its status (no model / bad prompt type)
                async with s.post(f"{url}/v1/completions", json={"prompt": 5}) as r:
                    assert r.status in (400, 404), r.status
            # chunked request body + Expect: 100-continue over a raw socket
            payload = json.dumps({"model": "m", "prompt": "chunked", "max_tokens": 2}).encode()
            req = (b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                   b"Transfer-Encoding: chunked\r\n\r\n" + b"%x\r\n" % 10 + payload[:10] + b"\r\n" +
                   b"%x\r\n" % (len(payload) - 10) + payload[10:] + b"\r\n0\r\n\r\n")
            resp = await _raw(port, req)
            assert resp.startswith(b"HTTP/1.1 200"), resp[:200]
            assert seen[-1]["body"]["prompt"] == "chunked"
            # the same body delivered in small pieces (incremental chunked parse)
            r, w = await asyncio.open_connection("127.0.0.1", port)
            for i in range(0, len(req), 7):
                w.write(req[i:i + 7])
                await w.drain()
                await asyncio.sleep(0.002)
            resp = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
            assert resp.startswith(b"HTTP/1.1 200"), resp[:200]
            w.close()
            # request smuggling shapes are refused (RFC 9112): whitespace before
            # the colon, bare CR inside a value, an obs-fold continuation line
            for bad in (b"Content-Length : 5\r\n", b"X-A: a\rb\r\n", b"X-A: a\r\n folded\r\n",
                        b"Transfer-Encoding\t: chunked\r\n"):
                resp = await _raw(port, b"POST /v1/completions HTTP/1.1\r\nHost: x\r\n" + bad +
                                  b"Content-Length: 2\r\n\r\n{}", read_until=b"\r\n\r\n")
                assert resp.startswith(b"HTTP/1.1 400"), (bad, resp[:200])
            # a chunked body past the 256 MB cap is a 413 (not unbounded buffering)
            resp = await _raw(port, b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
                              b"%x\r\n" % (300 << 20) + b"x" * 1024, read_until=b"\r\n\r\n")
            assert resp.startswith(b"HTTP/1.1 413"), resp[:200]
            r, w = await asyncio.open_connection("127.0.0.1", port)
            w.write(b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                    b"Expect: 100-continue\r\nContent-Length: %d\r\n\r\n" % len(payload))
            await w.drain()
            first = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
            assert first.startswith(b"HTTP/1.1 100"), first
            w.write(payload)
            await w.drain()
            rest = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
            assert rest.startswith(b"HTTP/1.1 200"), rest
            w.close()
            # a client that drops a slow stream: the decision is completed (nothing left open)
            r, w = await asyncio.open_connection("127.0.0.1", port)
            slow = json.dumps({"model": "m", "prompt": "slow", "max_tokens": 50, "stream": True, "delay": 0.05}).encode()
            w.write(b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                    b"Content-Length: %d\r\n\r\n" % len(slow) + slow)
            await w.drain()
            await asyncio.wait_for(r.readuntil(b"data: "), 5)
            assert srv.open
            w.close()
            for _ in range(100):
                if not srv.open:
                    break
                await asyncio.sleep(0.02)
            assert not srv.open
            assert all(v == 0 for v in epp.ctx.inflight_requests.values()), epp.ctx.inflight_requests
            # prefix affinity across the relay's threads: the sims join, the echo leaves
            for i, (_, _, p) in enumerate(sims):
                await store.add(endpoints_from_yaml({"endpoints": [{"name": f"s{i}", "address": "127.0.0.1",
                                                                     "port": p}]})[0])
            await store.remove(f"127.0.0.1:{eport}")
            await asyncio.sleep(0.7)  # the relay's state poll (0.5 s) picks up the endpoint list
            long = "lorem ipsum dolor sit amet " * 100
            n_before = [eng.metrics.prompt_tokens.labels("m")._value.get() for (_, eng, _) in sims]
            async with aiohttp.ClientSession() as s:
                for i in range(9):
                    async with aiohttp.ClientSession() as s2:  # new connections spread over the threads
                        async with s2.post(f"{url}/v1/completions", json={"model": "m", "prompt": long + f"q{i}",
                                                                          "max_tokens": 2}) as r:
                            assert r.status == 200
                            await r.read()
                # concurrent streams
                async def one(i):
                    async with s.post(f"{url}/v1/completions", json={"model": "m", "prompt": f"p{i}",
                                                                     "max_tokens": 4, "stream": True}) as r:
                        return r.status, await r.read()
                res = await asyncio.gather(*(one(i) for i in range(48)))
                assert all(st == 200 and b.strip().endswith(b"[DONE]") for st, b in res)
            per = [eng.metrics.prompt_tokens.labels("m")._value.get() - b
                   for (_, eng, _), b in zip(sims, n_before)]
            assert sum(1 for v in per if v > 2000) == 1, per
            # EPP gone: FailClose -> 503
            await srv.stop()
            relay.terminate()
            relay.wait(5)
            relay2 = spawn(str(tmp_path / "nobody.sock"), "127.0.0.1", port, 1, "FailClose")
            try:
                await asyncio.sleep(0.3)
                resp = await _raw(port, b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Length: 2\r\n\r\n{}",
                                  read_until=b"}}")
                assert resp.startswith(b"HTTP/1.1 503"), resp[:200]
                assert b"endpoint picker failed" in resp
                resp = await _raw(port, b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n", read_until=b"connecting")
                assert resp.startswith(b"HTTP/1.1 503")
            finally:
                relay2.terminate()
                relay2.wait(5)
        finally:
            if relay.poll() is None:
                relay.terminate()
                relay.wait(5)
            await epp.stop()
            await engine.cleanup()
            for r_, _, _ in sims:
                await r_.cleanup()
    asyncio.run(main())


def test_native_relay_dead_endpoint_502(tmp_path):
    async def main():
        store = EndpointStore()
        epp = EPP(BASE, store, ControlPlane())
        dead = _free_port()
        await store.add(endpoints_from_yaml({"endpoints": [{"name": "d", "address": "127.0.0.1", "port": dead}]})[0])
        await epp.start()
        uds = str(tmp_path / "epp.sock")
        srv = EppServer(epp)
        await srv.start(uds)
        port = _free_port()
        relay = spawn(uds, "127.0.0.1", port, 1, "FailClose")
        try:
            await _up(port, relay)
            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{port}/v1/completions",
                                  json={"model": "m", "prompt": "x", "max_tokens": 2}) as r:
                    assert r.status == 502
                    assert "failed" in (await r.json())["error"]["message"]
            await asyncio.sleep(0.1)
            assert not srv.open
        finally:
            relay.terminate()
            relay.wait(5)
            await srv.stop()
            await epp.stop()
    asyncio.run(main())


def test_native_relay_bad_epp_frame_fails_over(tmp_path):
    """an EPP frame that does not decode must not leave its pick
    pending forever - the relay treats it as a lost EPP (FailClose -> 503)."""
    import struct

    import msgpack

    async def main():
        uds = str(tmp_path / "bad.sock")

        async def serve(reader, writer):
            try:
                while True:
                    n = struct.unpack(">I", await reader.readexactly(4))[0]
                    m = msgpack.unpackb(await reader.readexactly(n), raw=False)
                    if m.get("op") == "state":
                        out = msgpack.packb({"id": m["id"], "eps": ["127.0.0.1:9"], "health": [200, "ok"]})
                    elif m.get("op") == "pick":
                        out = b"\xc1"  # the one byte msgpack never uses
                    else:
                        continue
                    writer.write(struct.pack(">I", len(out)) + out)
                    await writer.drain()
            except (asyncio.IncompleteReadError, ConnectionError):
                pass

        srv = await asyncio.start_unix_server(serve, uds)
        port = _free_port()
        relay = spawn(uds, "127.0.0.1", port, 1, "FailClose")
        try:
            await _up(port, relay)
            t0 = time.monotonic()
            resp = await _raw(port, b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Length: 2\r\n\r\n{}",
                              read_until=b"}}", timeout=10)
            assert resp.startswith(b"HTTP/1.1 503"), resp[:200]
            assert time.monotonic() - t0 < 5
        finally:
            relay.terminate()
            relay.wait(5)
            srv.close()
    asyncio.run(main())
