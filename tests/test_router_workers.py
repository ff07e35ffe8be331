"""Multi-worker router data plane (llmd_amd/router/workers.py): N proxy
workers relay streams, one EPP process owns the scheduling state.

* in one event loop: two WorkerProxy front-ends over one EppServer - every
  request is answered, prefix affinity holds ACROSS workers (one prefix index),
  EPP rejections keep their status and dropped-reason header, in-flight
  accounting returns to zero, a worker that disconnects has its open decisions
  completed;
* as processes: ``python -m llmd_amd.router.proxy --workers 2`` (SO_REUSEPORT)
  serves concurrent streaming requests and the EPP's /metrics counts them all.
"""
import asyncio
import json
import os
import socket
import subprocess
import sys
import time

import aiohttp
import pytest

from llmd_amd.router.api import ControlPlane
from llmd_amd.router.datalayer import EndpointStore, endpoints_from_yaml
from llmd_amd.router.epp import EPP
from llmd_amd.router.workers import EppClient, EppServer, WorkerProxy
from llmd_amd.sim.server import start_sim
from tests.test_router_e2e import BASE, _post, _serve

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_workers_share_one_epp(tmp_path):
    async def main():
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.0005) for _ in range(4)]
        eps = [{"name": f"s{i}", "address": "127.0.0.1", "port": p} for i, (_, _, p) in enumerate(sims)]
        store = EndpointStore()
        epp = EPP(BASE, store, ControlPlane())
        for e in endpoints_from_yaml({"endpoints": eps}):
            await store.add(e)
        await epp.start()
        uds = str(tmp_path / "epp.sock")
        srv = EppServer(epp)
        await srv.start(uds)
        fronts = []
        for _ in range(2):
            runner, port = await _serve(WorkerProxy(EppClient(uds, state_period=0.05), "FailClose").app())
            fronts.append((runner, port))
        long = "lorem ipsum dolor sit amet " * 100
        async with aiohttp.ClientSession() as s:
            # health through a worker reflects the EPP's endpoints
            async with s.get(f"http://127.0.0.1:{fronts[0][1]}/health") as r:
                assert r.status == 200
            # alternate workers: one prefix index -> every request on the same endpoint
            for i in range(8):
                port = fronts[i % 2][1]
                st, body, _ = await _post(s, f"http://127.0.0.1:{port}/v1/completions",
                                          {"model": "m", "prompt": long + f"q{i}", "max_tokens": 2})
                assert st == 200 and json.loads(body)["usage"]["completion_tokens"] == 2
            per = [eng.metrics.prompt_tokens.labels("m")._value.get() for (_, eng, _) in sims]
            assert sum(1 for v in per if v > 0) == 1, per
            # concurrent streams through both workers
            async def one(i):
                port = fronts[i % 2][1]
                st, body, _ = await _post(s, f"http://127.0.0.1:{port}/v1/completions",
                                          {"model": "m", "prompt": f"p{i}", "max_tokens": 6, "stream": True,
                                           "stream_options": {"include_usage": True}})
                return st, body
            res = await asyncio.gather(*(one(i) for i in range(40)))
            assert all(st == 200 and body.strip().endswith(b"[DONE]") for st, body in res)
            # an EPP rejection keeps its status through the worker (unknown path body -> 400)
            st, _, _ = await _post(s, f"http://127.0.0.1:{fronts[1][1]}/v1/completions", {"prompt": 5})
            assert st in (400, 404), st
        await asyncio.sleep(0.05)
        assert not srv.open
        assert all(v == 0 for v in epp.ctx.inflight_requests.values()), epp.ctx.inflight_requests
        text = epp.render_metrics().decode()
        assert "inference_objective_request_total" in text
        # a worker that goes away mid-request: its open decision is completed by the EPP
        c = EppClient(uds)
        await c.start()
        d = await c.handle("/v1/completions", json.dumps({"model": "m", "prompt": "x"}).encode(), {})
        key = d.endpoint.key
        assert srv.open and epp.ctx.inflight_requests.get(key, 0) >= 1
        await c.stop()
        for _ in range(50):
            if not srv.open:
                break
            await asyncio.sleep(0.02)
        assert not srv.open and epp.ctx.inflight_requests.get(key, 0) == 0
        for r, _ in fronts:
            await r.cleanup()
        await srv.stop()
        await epp.stop()
        for r, _, _ in sims:
            await r.cleanup()
    asyncio.run(main())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_router_process_with_workers():
    async def main():
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.0005) for _ in range(3)]
        port, mport = _free_port(), _free_port()
        eps = ",".join(f"127.0.0.1:{p}" for (_, _, p) in sims)
        proc = subprocess.Popen([sys.executable, "-m", "llmd_amd.router.proxy", "--workers", "2", "--port", str(port),
                                 "--metrics-port", str(mport), "--endpoints", eps], cwd=ROOT,
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        try:
            async with aiohttp.ClientSession() as s:
                for _ in range(300):
                    try:
                        async with s.get(f"http://127.0.0.1:{port}/health") as r:
                            if r.status == 200:
                                break
                    except aiohttp.ClientError:
                        pass
                    await asyncio.sleep(0.1)
                else:
                    raise AssertionError("router workers never became healthy")

                async def one(i):
                    return await _post(s, f"http://127.0.0.1:{port}/v1/completions",
                                       {"model": "m", "prompt": f"hello {i}", "max_tokens": 4, "stream": True})
                res = await asyncio.gather(*(one(i) for i in range(60)))
                assert all(st == 200 for st, _, _ in res)
                await asyncio.sleep(0.3)
                async with s.get(f"http://127.0.0.1:{mport}/metrics") as r:
                    text = await r.text()
                tot = sum(float(l.split()[-1]) for l in text.splitlines()
                          if l.startswith("inference_objective_request_total"))
                assert tot == 60, tot
        finally:
            proc.terminate()
            try:
                proc.wait(10)
            except subprocess.TimeoutExpired:
                proc.kill()
            for r, _, _ in sims:
                await r.cleanup()
    asyncio.run(main())
