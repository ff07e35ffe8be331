"""Batch Gateway (C29) and Async Processor (C31) end-to-end over HTTP on CPU,
against the engine simulator: file upload/validation, job lifecycle, per-model
plans, tenant isolation, cancellation, crash recovery, GC; async queue
dispatch, gates, retries with backoff, deadlines."""
import asyncio
import json
import time

import aiohttp
from aiohttp import web

from llmd_amd.batch.async_processor import AsyncProcessor, BudgetGate, PrometheusGate, SortedSetQueue
from llmd_amd.batch.gateway import BatchGateway, validate_input
from llmd_amd.batch.store import Store
from llmd_amd.sim.server import start_sim


async def _serve(app):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def _jsonl(n, model="m", url="/v1/completions", start=0):
    return "\n".join(json.dumps({"custom_id": f"c{i}", "method": "POST", "url": url,
                                 "body": {"model": model, "prompt": f"hello {i}", "max_tokens": 3}})
                     for i in range(start, start + n)).encode()


async def _upload(s, base, data, tenant="t1"):
    fd = aiohttp.FormData()
    fd.add_field("purpose", "batch")
    fd.add_field("file", data, filename="in.jsonl")
    async with s.post(base + "/v1/files", data=fd, headers={"x-llm-d-tenant": tenant}) as r:
        assert r.status == 200
        return await r.json()


async def _wait_status(s, base, bid, want, tenant="t1", timeout=20):
    t0 = time.time()
    while time.time() - t0 < timeout:
        async with s.get(f"{base}/v1/batches/{bid}", headers={"x-llm-d-tenant": tenant}) as r:
            b = await r.json()
        if b["status"] in want:
            return b
        await asyncio.sleep(0.05)
    raise AssertionError(f"batch stuck in {b['status']}")


def test_validate_input():
    good = _jsonl(3)
    reqs, errs = validate_input(good, "/v1/completions", 10)
    assert len(reqs) == 3 and not errs
    bad = good + b"\n{not json}\n" + json.dumps({"custom_id": "c0", "url": "/v1/embeddings",
                                                "body": {}}).encode()
    _, errs = validate_input(bad, "/v1/completions", 10)
    codes = {e["code"] for e in errs}
    assert {"invalid_json_line", "duplicate_custom_id", "mismatched_url", "missing_model"} <= codes
    _, errs = validate_input(_jsonl(5), "/v1/completions", 4)
    assert errs[-1]["code"] == "too_many_requests"


def test_batch_gateway_lifecycle(tmp_path):
    async def main():
        sim_r, sim, sim_port = await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001)
        sim2_r, sim2, sim2_port = await start_sim(model="m2", prefill_tps=1e6, decode_step_s=0.001)
        gw = BatchGateway(Store(str(tmp_path / "bg")), f"http://127.0.0.1:{sim_port}",
                          model_gateways={"m2": f"http://127.0.0.1:{sim2_port}"},
                          global_concurrency=4, per_model_concurrency=2, poll_interval=0.02)
        runner, port = await _serve(gw.app())
        base = f"http://127.0.0.1:{port}"
        async with aiohttp.ClientSession() as s:
            data = _jsonl(6) + b"\n" + _jsonl(4, model="m2", start=100)
            f = await _upload(s, base, data)
            assert f["purpose"] == "batch" and f["bytes"] == len(data)
            async with s.post(base + "/v1/batches", json={"input_file_id": f["id"], "endpoint": "/v1/completions",
                                                          "completion_window": "24h"},
                              headers={"x-llm-d-tenant": "t1"}) as r:
                b = await r.json()
            assert b["status"] == "validating" and b["request_counts"]["total"] == 10
            b = await _wait_status(s, base, b["id"], ("completed", "failed"))
            assert b["status"] == "completed", b
            assert b["request_counts"] == {"total": 10, "completed": 10, "failed": 0}
            async with s.get(f"{base}/v1/files/{b['output_file_id']}/content",
                             headers={"x-llm-d-tenant": "t1"}) as r:
                lines = [json.loads(x) for x in (await r.text()).splitlines()]
            assert sorted(x["custom_id"] for x in lines) == sorted([f"c{i}" for i in range(6)] +
                                                                   [f"c{i}" for i in range(100, 104)])
            assert all(x["response"]["status_code"] == 200 for x in lines)
            gen = lambda e: e.metrics.gen_tokens.labels(e.model)._value.get()  # noqa: E731
            assert gen(sim) == 18 and gen(sim2) == 12  # per-model gateways used
            # tenant isolation
            async with s.get(f"{base}/v1/batches/{b['id']}", headers={"x-llm-d-tenant": "t2"}) as r:
                assert r.status == 404
            async with s.get(f"{base}/v1/files", headers={"x-llm-d-tenant": "t2"}) as r:
                assert (await r.json())["data"] == []
            async with s.get(f"{base}/v1/batches", headers={"x-llm-d-tenant": "t1"}) as r:
                assert len((await r.json())["data"]) == 1
            # invalid input -> failed with errors
            f2 = await _upload(s, base, b'{"custom_id": "x"}')
            async with s.post(base + "/v1/batches", json={"input_file_id": f2["id"],
                                                          "endpoint": "/v1/completions"},
                              headers={"x-llm-d-tenant": "t1"}) as r:
                bb = await r.json()
            assert bb["status"] == "failed" and bb["errors"]["data"]
            # delete file
            async with s.delete(f"{base}/v1/files/{f2['id']}", headers={"x-llm-d-tenant": "t1"}) as r:
                assert (await r.json())["deleted"]
            async with s.get(f"{base}/metrics") as r:
                assert "batch_gateway_requests_total" in await r.text()
        await runner.cleanup()
        await sim_r.cleanup()
        await sim2_r.cleanup()

    asyncio.run(main())


def test_batch_cancel_and_recovery(tmp_path):
    async def main():
        sim_r, sim, sim_port = await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.02)
        store = Store(str(tmp_path / "bg"))
        gw = BatchGateway(store, f"http://127.0.0.1:{sim_port}", global_concurrency=1, per_model_concurrency=1,
                          poll_interval=0.02)
        runner, port = await _serve(gw.app())
        base = f"http://127.0.0.1:{port}"
        async with aiohttp.ClientSession() as s:
            f = await _upload(s, base, _jsonl(40))
            async with s.post(base + "/v1/batches", json={"input_file_id": f["id"],
                                                          "endpoint": "/v1/completions"},
                              headers={"x-llm-d-tenant": "t1"}) as r:
                b = await r.json()
            await _wait_status(s, base, b["id"], ("in_progress",))
            await asyncio.sleep(0.2)
            async with s.post(f"{base}/v1/batches/{b['id']}/cancel", headers={"x-llm-d-tenant": "t1"}) as r:
                assert (await r.json())["status"] == "cancelling"
            b = await _wait_status(s, base, b["id"], ("cancelled",))
            assert 0 < b["request_counts"]["completed"] < 40
            assert b["output_file_id"]
        await runner.cleanup()
        # crash recovery: a job marked in_progress without output is re-enqueued
        store.put_batch("t1", {"id": "batch_x", "status": "in_progress", "expires_at": time.time() + 100,
                               "input_file_id": f["id"], "endpoint": "/v1/completions",
                               "request_counts": {"total": 40, "completed": 3, "failed": 0}})
        gw2 = BatchGateway(store, f"http://127.0.0.1:{sim_port}")
        gw2.recover()
        assert store.get_batch("t1", "batch_x")["status"] == "validating" and store.queue_len() == 1
        # GC removes terminal jobs past retention
        gw2.job_retention_s = 0
        gw2.gc(now=time.time() + 10)
        assert store.get_batch("t1", b["id"]) is None
        await sim_r.cleanup()

    asyncio.run(main())


def test_async_processor_retries_and_deadlines(tmp_path):
    async def main():
        calls = {"n": 0}

        async def flaky(req):
            calls["n"] += 1
            body = await req.json()
            if body.get("prompt") == "flaky" and calls["n"] < 3:
                return web.json_response({"error": {"message": "busy"}}, status=503)
            if body.get("prompt") == "bad":
                return web.json_response({"error": {"message": "bad"}}, status=400)
            return web.json_response({"choices": [{"text": "ok"}], "echo": body.get("prompt")})

        app = web.Application()
        app.router.add_post("/v1/completions", flaky)
        runner, port = await _serve(app)
        mq = SortedSetQueue(str(tmp_path / "mq.db"))
        proc = AsyncProcessor(mq, f"http://127.0.0.1:{port}", workers=4, base_backoff=0.01)
        now = time.time()
        mq.zadd(now + 30, json.dumps({"id": "a", "payload": {"prompt": "flaky"}, "deadline": now + 30}))
        mq.zadd(now + 30, json.dumps({"id": "b", "payload": {"prompt": "bad"}, "deadline": now + 30}))
        mq.zadd(now - 1, json.dumps({"id": "c", "payload": {"prompt": "late"}, "deadline": now - 1}))
        mq.zadd(now + 30, json.dumps({"id": "d", "payload": {"prompt": "fine"}, "deadline": now + 30}))
        await proc.start()
        res = {}
        t0 = time.time()
        while len(res) < 4 and time.time() - t0 < 10:
            r = mq.rpop_result()
            if r is None:
                await asyncio.sleep(0.02)
                continue
            d = json.loads(r)
            res[d["id"]] = d
        await proc.stop()
        assert res["a"]["status_code"] == 200 and proc.m_retry._value.get() >= 1
        assert res["b"]["status_code"] == 400  # fatal: not retried
        assert res["c"]["payload"]["error"]["code"] == "deadline_exceeded"
        assert res["d"]["payload"]["echo"] == "fine"
        # budget gate: closed gate sheds at the deadline
        gate = BudgetGate(0)
        proc2 = AsyncProcessor(mq, f"http://127.0.0.1:{port}", gate=gate, workers=1)
        await proc2.start()
        await proc2.handle({"id": "e", "payload": {"prompt": "x"}, "deadline": time.time() + 0.2})
        assert json.loads(mq.rpop_result())["payload"]["error"]["code"] == "deadline_exceeded"
        gate.value = 5
        await proc2.handle({"id": "f", "payload": {"prompt": "x"}, "deadline": time.time() + 5})
        assert json.loads(mq.rpop_result())["status_code"] == 200
        await proc2.stop()
        await runner.cleanup()

    asyncio.run(main())


def test_prometheus_saturation_gate():
    async def main():
        sim_r, sim, port = await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001)
        g = PrometheusGate([f"http://127.0.0.1:{port}"], "saturation", max_running=8)
        assert await g.budget() == 8  # idle pool: open
        g2 = PrometheusGate(["http://127.0.0.1:1"], "budget")
        assert await g2.budget() == 0  # unreachable pod counts as saturated
        await g.close()
        await g2.close()
        await sim_r.cleanup()

    asyncio.run(main())
