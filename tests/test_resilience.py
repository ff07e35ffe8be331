"""Inference Resilience Operator (llmd_amd/resilience/operator.py; SURVEY C43,
proposals/inference-resilience-operator.md:66-256): the three recovery tracks,
failed recovery, engine-initiated transient faults over the ``vllm_fault``
channel, and the real API server's ``/fault_tolerance`` surface on CPU."""
import asyncio
import os
import socket

import pytest
import yaml
from aiohttp import web

from llmd_amd.resilience.operator import (LLMDEngineAdapter, RecoveryRequest, RecoveryStore,
                                          ResilienceOperator, main)
from llmd_amd.serving.kv_events import KVEventPublisher


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeEngine:
    """An engine's /fault_tolerance surface that records the operator's calls."""

    def __init__(self):
        self.calls = []
        self.paused = False
        self.faulted = False
        self.heal_on_retry = True

    def app(self):
        app = web.Application()

        async def status(_):
            st = "faulted" if self.faulted else ("paused" if self.paused else "healthy")
            return web.json_response({"status": st, "faults": [{"kind": "x"}] if self.faulted else []})

        async def apply(req):
            act = (await req.json())["action"]
            self.calls.append(act)
            if act == "pause":
                self.paused = True
            elif act in ("resume", "retry"):
                self.paused = False
                if act == "retry" and self.heal_on_retry:
                    self.faulted = False
            return web.json_response({"applied": act})

        app.router.add_get("/fault_tolerance/status", status)
        app.router.add_post("/fault_tolerance/apply", apply)
        return app


async def _start(app, port):
    runner = web.AppRunner(app)
    await runner.setup()
    await web.TCPSite(runner, "127.0.0.1", port).start()
    return runner


async def _until(cond, timeout=10.0):
    t = asyncio.get_running_loop().time() + timeout
    while not cond():
        if asyncio.get_running_loop().time() > t:
            raise AssertionError("condition not reached")
        await asyncio.sleep(0.05)


def _eps_file(tmp_path, ports):
    p = str(tmp_path / "endpoints.yaml")
    with open(p, "w") as f:
        yaml.safe_dump({"endpoints": [{"name": f"e{port}", "address": "127.0.0.1", "port": port}
                                      for port in ports]}, f)
    return p


def _routed(path):
    with open(path) as f:
        return sorted(e["port"] for e in yaml.safe_load(f)["endpoints"])


def test_recovery_request_schema(tmp_path):
    st = RecoveryStore(str(tmp_path / "rr"))
    rr = st.create({"metadata": {"name": "gpu3"}, "spec": {"nodeName": "n0", "deviceID": 3,
                                                            "requestedAction": "RESET_DEVICE", "errorCode": "XGMI_48"}})
    assert rr.track == "A" and rr.phase == "Pending" and rr.active
    with pytest.raises(ValueError):
        st.create({"spec": {"nodeName": "n0", "requestedAction": "FORMAT_DISK"}})
    with pytest.raises(FileExistsError):
        st.create({"metadata": {"name": "gpu3"}, "spec": {"nodeName": "n0", "requestedAction": "REBOOT_NODE"}})
    st.set_phase("gpu3", "InProgress")
    back = RecoveryRequest.from_obj(rr.to_obj())
    assert back.device_id == 3 and back.error_code == "XGMI_48"
    assert st.get("gpu3").phase == "InProgress"
    # CLI: the infrastructure side
    main(["request", "--store", st.root, "--node", "n0", "--action", "REPLACE_NODE", "--name", "node"])
    main(["complete", "--store", st.root, "node", "--failed"])
    assert st.get("node").phase == "Failed" and st.get("node").track == "C"


def test_tracks_failed_and_transient(tmp_path):
    async def run():
        engs = [FakeEngine() for _ in range(4)]
        ports = [_free_port() for _ in engs]
        runners = [await _start(e.app(), p) for e, p in zip(engs, ports)]
        eps = _eps_file(tmp_path, ports)
        cfg = {"recoveryRequestsDir": str(tmp_path / "rr"), "endpointsFile": eps, "interval": 0.05,
               "recoverTimeout": 2.0, "maxRetries": 2, "retryWindow": 60,
               "engines": [{"name": "e0", "url": f"http://127.0.0.1:{ports[0]}", "nodeName": "n0", "devices": [0]},
                           {"name": "e1", "url": f"http://127.0.0.1:{ports[1]}", "nodeName": "n0", "devices": [1]},
                           # a wide-EP pair: DP ranks in lockstep share one fate
                           {"name": "e2", "url": f"http://127.0.0.1:{ports[2]}", "nodeName": "n1", "devices": [0],
                            "group": "ep"},
                           {"name": "e3", "url": f"http://127.0.0.1:{ports[3]}", "nodeName": "n1", "devices": [1],
                            "group": "ep"}]}
        op = ResilienceOperator(cfg)
        st = op.store
        try:
            # Track A: pause the device's engine only, resume on Completed
            st.create({"metadata": {"name": "a"}, "spec": {"nodeName": "n0", "deviceID": 0,
                                                           "requestedAction": "RESET_DEVICE"}})
            await op.reconcile()
            a = st.get("a")
            assert a.iro_state == "EnginePaused" and a.conditions["EngineReadyForRecovery"] == "True"
            assert engs[0].calls == ["pause"] and engs[1].calls == []
            await op.reconcile()  # idempotent while the infrastructure works
            assert engs[0].calls == ["pause"]
            st.set_phase("a", "Completed")
            await op.reconcile()
            assert st.get("a").iro_state == "Recovered" and engs[0].calls == ["pause", "resume"]
            assert _routed(eps) == sorted(ports)

            # Track C on an independent replica: out of routing, back after replacement
            st.create({"metadata": {"name": "c"}, "spec": {"nodeName": "n0", "deviceID": 1,
                                                           "requestedAction": "REPLACE_NODE"}})
            await op.reconcile()
            c = st.get("c")
            assert c.iro_state == "EngineScaledDown" and ports[1] not in _routed(eps)
            assert [e["port"] for e in c.removed_endpoints] == [ports[1]]
            st.set_phase("c", "Completed")
            await op.reconcile()
            assert st.get("c").iro_state == "Recovered" and _routed(eps) == sorted(ports)

            # Track C on a lockstep EP group: every rank pauses (the EP world cannot shrink)
            st.create({"metadata": {"name": "g"}, "spec": {"nodeName": "n1", "deviceID": 1,
                                                           "requestedAction": "REPLACE_NODE"}})
            await op.reconcile()
            assert st.get("g").iro_state == "EnginePaused" and sorted(st.get("g").engines) == ["e2", "e3"]
            assert engs[2].calls == ["pause"] and engs[3].calls == ["pause"]
            # infrastructure recovery failed: the group stays out of routing
            st.set_phase("g", "Failed")
            await op.reconcile()
            g = st.get("g")
            assert g.iro_state == "Degraded" and _routed(eps) == sorted(ports[:2])

            # engine-initiated transient fault: retry, no request involved
            engs[0].faulted = True
            await op.reconcile()
            await _until(lambda: "retry" in engs[0].calls)
            assert not engs[0].faulted
            # a fault that keeps coming back: after maxRetries the engine leaves routing
            engs[1].heal_on_retry = False
            for _ in range(4):
                engs[1].faulted = True
                op._faulted.discard("e1")
                await op.reconcile()
            assert engs[1].calls.count("retry") == 2 and "e1" in op.degraded
            assert ports[1] not in _routed(eps)
            op.readmit("e1")
            assert ports[1] in _routed(eps)
            text = op.render_metrics()
            assert 'iro_engine_actions_total{engine="e0",action="pause"} 1' in text
            assert 'requested_action="REPLACE_NODE"' in text
        finally:
            for r in runners:
                await r.cleanup()

    asyncio.run(run())


def test_fault_events_channel_and_http_api(tmp_path):
    """vllm_fault events from the engine's publisher reach the operator without
    polling; RecoveryRequests created / completed over the operator's HTTP API."""
    import aiohttp

    async def run():
        eng = FakeEngine()
        eport, oport = _free_port(), _free_port()
        runner = await _start(eng.app(), eport)
        pub = KVEventPublisher("tcp://127.0.0.1:0", "kv@x", 16)
        cfg = {"recoveryRequestsDir": str(tmp_path / "rr"), "interval": 0.05, "pollEngineStatus": False,
               "engines": [{"name": "e0", "url": f"http://127.0.0.1:{eport}", "nodeName": "n0", "devices": [0],
                            "faultEvents": f"tcp://127.0.0.1:{pub.port}"}]}
        op = ResilienceOperator(cfg).start()
        orun = await _start(op.app(), oport)
        try:
            await _until(lambda: op._subs[0].connected.is_set())
            pub.publish_batch({"events": [{"type": "vllm_fault", "action": "detected", "faults": [{"kind": "x"}]}]},
                              topic="fault@m")
            await _until(lambda: eng.calls == ["retry"])
            base = f"http://127.0.0.1:{oport}"
            async with aiohttp.ClientSession() as s:
                async with s.post(base + "/apis/recoveryrequests",
                                  json={"metadata": {"name": "r1"},
                                        "spec": {"nodeName": "n0", "requestedAction": "REBOOT_NODE"}}) as r:
                    assert r.status == 201
                async with s.post(base + "/apis/recoveryrequests", json={"spec": {"nodeName": "n0"}}) as r:
                    assert r.status == 400
                await _until(lambda: eng.calls[-1:] == ["pause"])
                # a fault event for an engine a request already covers is not retried
                pub.publish_batch({"events": [{"type": "vllm_fault", "action": "detected",
                                               "faults": [{"kind": "x"}]}]}, topic="fault@m")
                await asyncio.sleep(0.3)
                assert eng.calls == ["retry", "pause"]
                async with s.patch(base + "/apis/recoveryrequests/r1/status",
                                   json={"status": {"phase": "Completed"}}) as r:
                    assert r.status == 200
                await _until(lambda: op.store.get("r1").iro_state == "Recovered")
                async with s.get(base + "/apis/recoveryrequests/r1") as r:
                    body = await r.json()
                assert body["status"]["conditions"] == [{"type": "EngineReadyForRecovery", "status": "True"}]
                async with s.get(base + "/metrics") as r:
                    assert 'iro_recovery_requests{phase="Completed",iro_state="Recovered"' in await r.text()
        finally:
            await op.stop()
            await orun.cleanup()
            await runner.cleanup()
            pub.close()

    asyncio.run(run())


def test_operator_against_api_server(tmp_path):
    """The LLMD adapter against the real API server (tiny model on CPU): the
    server's fault monitor publishes ``vllm_fault`` when its fault set changes,
    and pause / resume / retry go through ``/fault_tolerance/apply``."""
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.serving.api_server import build_server

    os.environ["LLMD_FAULT_POLL_S"] = "0.05"

    async def run():
        kport, sport = _free_port(), _free_port()
        cfg = EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                                  max_num_batched_tokens=128, max_num_seqs=4, max_model_len=512,
                                  enforce_eager=True)
        cfg.kv_events_config = {"enable_kv_cache_events": True, "endpoint": f"tcp://127.0.0.1:{kport}"}
        srv = build_server(cfg)
        runner = await _start(srv.app(), sport)
        events = []
        from llmd_amd.serving.kv_events import KVEventSubscriber

        sub = KVEventSubscriber(f"tcp://127.0.0.1:{kport}", lambda t, b: events.extend(b["events"]),
                                topic_filter="fault@").start()
        ad = LLMDEngineAdapter("e0", "n0", [0], [{"address": "127.0.0.1", "port": sport}],
                               url=f"http://127.0.0.1:{sport}")
        try:
            await _until(lambda: sub.connected.is_set())
            assert (await ad.status())["status"] == "healthy"
            await ad.pause()
            assert (await ad.status())["status"] == "paused"
            await ad.retry()
            assert (await ad.status())["status"] == "healthy"
            srv.aeng.dead = RuntimeError("HIP error: device lost")  # what the engine loop records
            await _until(lambda: any(e.get("action") == "detected" for e in events))
            assert (await ad.status())["status"] == "faulted"
            srv.aeng.dead = None
            await _until(lambda: any(e.get("action") == "cleared" for e in events))
        finally:
            await sub.stop()
            await runner.cleanup()
            srv.aeng.shutdown()
            srv.kv_event_publisher.close()
            os.environ.pop("LLMD_FAULT_POLL_S", None)

    asyncio.run(run())


def test_launcher_generates_rank_topology(tmp_path):
    """``services: [{type: iro}]``: the launcher writes the operator's rank
    topology map from its own plan (devices per DP rank, one lockstep group per
    wide-EP replica, fault-event ports = the ranks' KV-event ports)."""
    from llmd_amd.launch import plan

    topo = {"model": "deepseek-v3", "gpus": 8, "node_name": "mi355x-0",
            "roles": [{"name": "prefill-decode", "dp": 4, "port": 8200, "kv_events": True,
                       "args": ["--enable-expert-parallel"]},
                      {"name": "decode", "replicas": 2, "tp": 2, "port": 8300, "kv_transfer": False}],
            "services": [{"type": "iro"}]}
    specs, doc = plan(topo, str(tmp_path))
    svc = specs[-1]
    assert svc.cmd[2] == "llmd_amd.resilience.operator" and svc.health == "/healthz" and svc.port == 8480
    with open(tmp_path / "iro-config.yaml") as f:
        conf = yaml.safe_load(f)
    engines = {e["name"]: e for e in conf["engines"]}
    assert sorted(engines) == ["decode-0", "decode-1", "prefill-decode-0-dp0", "prefill-decode-0-dp1",
                               "prefill-decode-0-dp2", "prefill-decode-0-dp3"]
    assert engines["prefill-decode-0-dp2"]["devices"] == [2] and engines["prefill-decode-0-dp2"]["group"] == \
        "prefill-decode-0"
    assert engines["prefill-decode-0-dp3"]["faultEvents"] == "tcp://127.0.0.1:5559"
    assert engines["decode-1"]["devices"] == [6, 7] and "group" not in engines["decode-1"]
    op = ResilienceOperator(conf)
    rr = RecoveryRequest.from_obj({"kind": "RecoveryRequest", "metadata": {"name": "x"},
                                   "spec": {"nodeName": "mi355x-0", "deviceID": 1,
                                            "requestedAction": "RESET_DEVICE"}})
    assert sorted(a.name for a in op.affected(rr)) == [f"prefill-decode-0-dp{r}" for r in range(4)]
    rr.device_id = 7
    assert [a.name for a in op.affected(rr)] == ["decode-1"]
