"""Multi-worker router data plane.

The reference runs its standalone proxy with ``--concurrency 8`` worker threads
in front of one EPP (guides/no-kubernetes-deployment/README.md:205-218,
guides/recipes/router/base.values.yaml:30-40). One Python process relaying every
token of every stream saturates around 800-900 req/s and adds hundreds of ms of
TTFT at 256 streams (profiles/router_overhead.txt B), so here:

* ONE EPP process owns all scheduling state (data layer, prefix index, flow
  control, predictor, metrics) - single writer, exactly the in-process EPP;
* N proxy WORKER processes accept client connections on the same port
  (SO_REUSEPORT: the kernel spreads connections over them), ask the EPP for a
  decision over a local Unix socket, and relay the response stream themselves.

Wire protocol (UDS, one multiplexed connection per worker): 4-byte big-endian
length + msgpack map.
  worker -> EPP  {"op": "pick", "id", "path", "headers", "body"}
  EPP -> worker  {"id", "d": {tok, endpoint, headers, body, request_id, stream}}
                 or {"id", "err": {status, msg, reason}} (SchedulingError: the
                 client sees the same status / dropped-reason headers)
  worker -> EPP  {"op": "hdr", "tok", "status", "headers"}      (no reply)
  worker -> EPP  {"op": "chunk", "tok", "chunk", "t"}            (only if a
                 response processor overrides on_response_chunk)
  worker -> EPP  {"op": "done", "tok", "info"}                   (no reply)
  worker -> EPP  {"op": "state", "id"} -> {"id", "eps", "health", "chunks"}
  worker -> EPP  {"op": "metrics", "id"} -> {"id", "text"}
A decision's EPP-side state (the Decision object and its in-flight accounting)
stays in the EPP under ``tok`` until the worker reports ``done``, so response
hooks (prefix-cache confirmation, predictor training, SLO metrics, flow control)
run exactly as in the single-process proxy. A worker that dies has its open
decisions completed with status 502 so in-flight counters do not leak.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import os
import struct
import time
from dataclasses import dataclass, field
from typing import Optional

import msgpack
from aiohttp import web

from .plugins.base import ResponseProcessor
from .proxy import RouterProxy
from .types import SchedulingError

log = logging.getLogger("llmd.router.workers")

_LEN = struct.Struct(">I")


async def _read_frame(reader: asyncio.StreamReader) -> Optional[dict]:
    try:
        n = _LEN.unpack(await reader.readexactly(4))[0]
        return msgpack.unpackb(await reader.readexactly(n), raw=False)
    except (asyncio.IncompleteReadError, ConnectionResetError):
        return None


def _frame(msg: dict) -> bytes:
    b = msgpack.packb(msg, use_bin_type=True)
    return _LEN.pack(len(b)) + b


def _needs_chunks(epp) -> bool:
    """True if some response processor overrides on_response_chunk (workers then
    forward chunk timing to the EPP; the built-in plugins do not need it)."""
    base = ResponseProcessor.on_response_chunk
    return any(getattr(type(p), "on_response_chunk", base) is not base for p in epp.cfg.response_processors)


# ---------------------------------------------------------------- EPP side
class EppServer:
    """Serves an in-process EPP to proxy workers over a Unix socket."""

    def __init__(self, epp, elector=None):
        self.epp = epp
        self.elector = elector
        self.open: dict[int, tuple] = {}  # tok -> (Decision, owner connection id)
        self._tok = itertools.count(1)
        self._conn = itertools.count(1)
        self.server: Optional[asyncio.AbstractServer] = None
        self.chunks = _needs_chunks(epp)

    async def start(self, path: str):
        if os.path.exists(path):
            os.unlink(path)
        self.server = await asyncio.start_unix_server(self._serve, path=path)

    async def stop(self):
        if self.server is not None:
            self.server.close()
            await self.server.wait_closed()

    def _health(self) -> tuple[int, str]:
        if self.elector is not None and not self.elector.is_leader:
            return 503, "standby"
        return (200, "ok") if self.epp.store.all() else (503, "no endpoints")

    async def _serve(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        cid = next(self._conn)
        lock = asyncio.Lock()

        async def reply(msg):
            async with lock:
                writer.write(_frame(msg))
                await writer.drain()

        tasks = set()
        try:
            while True:
                msg = await _read_frame(reader)
                if msg is None:
                    break
                op = msg.get("op")
                if op == "pick":
                    t = asyncio.ensure_future(self._pick(msg, cid, reply))
                    tasks.add(t)
                    t.add_done_callback(tasks.discard)
                elif op == "done":
                    ent = self.open.pop(msg["tok"], None)
                    if ent is not None:
                        self.epp.on_response_complete(ent[0], msg.get("info") or {})
                elif op == "hdr":
                    ent = self.open.get(msg["tok"])
                    if ent is not None:
                        self.epp.on_response_headers(ent[0], msg["status"], msg.get("headers") or {})
                elif op == "chunk":
                    ent = self.open.get(msg["tok"])
                    if ent is not None:
                        self.epp.on_response_chunk(ent[0], msg["chunk"], msg["t"])
                elif op == "state":
                    st, txt = self._health()
                    await reply({"id": msg["id"], "eps": [e.key for e in self.epp.store.all()],
                                 "health": [st, txt], "chunks": self.chunks})
                elif op == "metrics":
                    await reply({"id": msg["id"], "text": self.epp.render_metrics()})
        finally:
            for t in list(tasks):
                t.cancel()
            # a dead worker: complete its open decisions so in-flight accounting does not leak
            for tok, (d, owner) in list(self.open.items()):
                if owner == cid:
                    self.open.pop(tok, None)
                    self.epp.on_response_complete(d, {"status": 502})
            writer.close()

    async def _pick(self, msg, cid, reply):
        try:
            d = await self.epp.handle(msg["path"], msg["body"], msg["headers"])
        except SchedulingError as e:
            await reply({"id": msg["id"], "err": {"status": e.status, "msg": str(e), "reason": e.reason}})
            return
        except Exception as e:  # noqa: BLE001 - the worker applies FailOpen / FailClose
            log.exception("EPP failure")
            await reply({"id": msg["id"], "err": {"status": -1, "msg": str(e), "reason": ""}})
            return
        tok = next(self._tok)
        self.open[tok] = (d, cid)
        await reply({"id": msg["id"], "d": {"tok": tok, "endpoint": d.endpoint.key, "headers": d.headers,
                                            "body": d.body, "request_id": d.req.request_id,
                                            "stream": bool(d.req.stream)}})


# ---------------------------------------------------------------- worker side
@dataclass
class _Ep:
    key: str


@dataclass
class _Req:
    request_id: str
    stream: bool


@dataclass
class RemoteDecision:
    tok: int
    endpoint: _Ep
    req: _Req
    headers: dict = field(default_factory=dict)
    body: Optional[bytes] = None


class _Store:
    def __init__(self, client: "EppClient"):
        self.client = client

    def all(self):
        return [_Ep(k) for k in self.client.eps]


class EppClient:
    """The EPP interface RouterProxy uses (handle / store / response hooks /
    render_metrics), served by a remote EppServer. One multiplexed connection."""

    class EppUnavailable(RuntimeError):
        pass

    def __init__(self, path: str, state_period: float = 0.5):
        self.path = path
        self.state_period = state_period
        self.reader = self.writer = None
        self.pending: dict[int, asyncio.Future] = {}
        self._ids = itertools.count(1)
        self.eps: list[str] = []
        self.health = (503, "connecting")
        self.chunks = False
        self.store = _Store(self)
        self._tasks: list[asyncio.Task] = []

    async def start(self):
        for i in range(200):  # the EPP process may still be starting
            try:
                self.reader, self.writer = await asyncio.open_unix_connection(self.path)
                break
            except (FileNotFoundError, ConnectionRefusedError):
                await asyncio.sleep(0.05)
        else:
            raise self.EppUnavailable(f"EPP socket {self.path} not reachable")
        self._tasks.append(asyncio.ensure_future(self._recv()))
        await self._refresh()
        self._tasks.append(asyncio.ensure_future(self._poll_state()))

    async def stop(self):
        for t in self._tasks:
            t.cancel()
        if self.writer is not None:
            self.writer.close()

    async def _recv(self):
        while True:
            msg = await _read_frame(self.reader)
            if msg is None:
                for f in self.pending.values():
                    if not f.done():
                        f.set_exception(self.EppUnavailable("EPP connection lost"))
                self.pending.clear()
                self.health = (503, "EPP connection lost")
                return
            f = self.pending.pop(msg.get("id"), None)
            if f is not None and not f.done():
                f.set_result(msg)

    def _send(self, msg: dict):
        self.writer.write(_frame(msg))

    async def _call(self, msg: dict) -> dict:
        i = next(self._ids)
        msg["id"] = i
        f = asyncio.get_running_loop().create_future()
        self.pending[i] = f
        self._send(msg)
        return await f

    async def _refresh(self):
        r = await self._call({"op": "state"})
        self.eps = r["eps"]
        self.health = tuple(r["health"])
        self.chunks = bool(r.get("chunks"))

    async def _poll_state(self):
        while True:
            await asyncio.sleep(self.state_period)
            try:
                await self._refresh()
            except self.EppUnavailable:
                return

    async def handle(self, path: str, body: bytes, headers) -> RemoteDecision:
        r = await self._call({"op": "pick", "path": path, "headers": dict(headers), "body": body})
        if "err" in r:
            e = r["err"]
            if e["status"] == -1:
                raise RuntimeError(e["msg"])
            raise SchedulingError(e["status"], e["msg"], e["reason"])
        d = r["d"]
        return RemoteDecision(d["tok"], _Ep(d["endpoint"]), _Req(d["request_id"], d["stream"]), d["headers"] or {},
                              d["body"])

    def on_response_headers(self, d, status: int, headers: dict):
        if isinstance(d, RemoteDecision):
            self._send({"op": "hdr", "tok": d.tok, "status": status, "headers": dict(headers)})

    def on_response_chunk(self, d, chunk: bytes, t: float):
        if self.chunks and isinstance(d, RemoteDecision):
            self._send({"op": "chunk", "tok": d.tok, "chunk": bytes(chunk), "t": t})

    def on_response_complete(self, d, info: dict):
        if isinstance(d, RemoteDecision):
            self._send({"op": "done", "tok": d.tok, "info": {k: v for k, v in info.items()
                                                            if isinstance(v, (int, float, str, dict, type(None)))}})

    def render_metrics(self) -> bytes:  # served by the EPP process's own metrics port
        return b""

    @property
    def active(self) -> bool:
        return self.health[1] != "standby"


class WorkerProxy(RouterProxy):
    """RouterProxy over an EppClient: health / standby state come from the EPP
    process; the response stream is relayed in this worker."""

    @property
    def active(self) -> bool:
        return self.epp.active

    async def health(self, req):
        st, txt = self.epp.health
        return web.Response(text=txt, status=st)


def worker_main(uds: str, host: str, port: int, failure_mode: str):
    """One proxy worker process: WorkerProxy over an EppClient, SO_REUSEPORT."""
    logging.basicConfig(level=logging.INFO)
    prox = WorkerProxy(EppClient(uds), failure_mode)
    app = prox.app()

    async def run():
        runner = web.AppRunner(app, access_log=None)
        await runner.setup()
        await web.TCPSite(runner, host, port, reuse_port=True).start()
        log.info("router worker %d listening on :%d", os.getpid(), port)
        while True:
            await asyncio.sleep(3600)

    asyncio.run(run())


def run_multi(epp, elector, host: str, port: int, metrics_port: int, workers: int, failure_mode: str,
              seed=None, grpc_port: int = 0, grpc_offset: int = 0, data_plane: str = "native"):
    """Parent process: the EPP (+ its metrics port, discovery, the h2c gRPC router)
    and an EppServer on a Unix socket; the data plane serves ``port``:
    ``native`` = one llmd-relay process with ``workers`` epoll threads
    (router/relay.py, csrc/relay/relay.cpp), ``python`` = ``workers`` aiohttp
    WorkerProxy processes. A data-plane process that exits is restarted; the
    parent exits non-zero if it cannot keep them up."""
    import multiprocessing as mp

    uds = f"/tmp/llmd-epp-{os.getpid()}-{port}.sock"
    ctx = mp.get_context("spawn")
    relay_bin = None
    if data_plane == "native":
        from .relay import relay_binary

        relay_bin = relay_binary()
        if relay_bin is None:
            log.warning("native relay unavailable: falling back to %d Python proxy workers", workers)

    async def run():
        if seed is not None:
            await seed()
        await epp.start()
        if elector is not None:
            elector.start()
        srv = EppServer(epp, elector)
        await srv.start(uds)

        async def metrics(req):
            return web.Response(body=epp.render_metrics(), content_type="text/plain")

        mapp = web.Application()
        mapp.router.add_get("/metrics", metrics)
        mr = web.AppRunner(mapp)
        await mr.setup()
        await web.TCPSite(mr, "0.0.0.0", metrics_port).start()
        if grpc_port:
            from .grpc_proxy import GrpcRouter, offset_target

            await GrpcRouter(epp, offset_target(grpc_offset)).start(grpc_port)
        if relay_bin is not None:
            from .relay import spawn

            relay = [spawn(uds, host, port, workers, failure_mode, relay_bin)]
            log.info("router: EPP pid %d, native relay pid %d with %d threads on :%d (metrics :%d)", os.getpid(),
                     relay[0].pid, workers, port, metrics_port)
            try:
                restarts = 0
                while True:
                    await asyncio.sleep(1.0)
                    if relay[0].poll() is not None:
                        restarts += 1
                        if restarts > 10:
                            raise SystemExit("router relay keeps dying")
                        log.warning("router relay exited (%s): restarting", relay[0].returncode)
                        relay[0] = spawn(uds, host, port, workers, failure_mode, relay_bin)
            finally:
                if relay[0].poll() is None:
                    relay[0].terminate()
                    try:
                        relay[0].wait(5)
                    except Exception:  # noqa: BLE001
                        relay[0].kill()
        procs = []
        for i in range(workers):
            p = ctx.Process(target=worker_main, args=(uds, host, port, failure_mode), daemon=True)
            p.start()
            procs.append(p)
        log.info("router: EPP pid %d, %d proxy workers on :%d (metrics :%d)", os.getpid(), workers, port,
                 metrics_port)
        restarts = 0
        while True:
            await asyncio.sleep(1.0)
            for i, p in enumerate(procs):
                if not p.is_alive():
                    restarts += 1
                    if restarts > 10 * workers:
                        raise SystemExit("router workers keep dying")
                    log.warning("router worker %d exited (%s): restarting", p.pid, p.exitcode)
                    q = ctx.Process(target=worker_main, args=(uds, host, port, failure_mode), daemon=True)
                    q.start()
                    procs[i] = q

    import signal

    def _term(*_):
        raise SystemExit(0)  # unwinds run(): the relay child is terminated in its finally

    signal.signal(signal.SIGTERM, _term)
    try:
        asyncio.run(run())
    finally:
        if os.path.exists(uds):
            os.unlink(uds)


__all__ = ["EppServer", "EppClient", "RemoteDecision", "WorkerProxy", "run_multi", "worker_main"]
