"""Active-passive HA by lease (SURVEY C08 EPP HA, configuration.md:455-459;
WVA --leader-elect, wva.md:397-400): one holder at a time, takeover on clean
release at once and on holder death after the lease duration, a stalled
leader steps down at its renew deadline; the router serves only on the
leader and its standby takes over over real HTTP; WVA standbys do not act."""
import asyncio
import os
import subprocess
import sys
import time

import aiohttp
import pytest

from llmd_amd.utils.leader import LeaseElector

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mk(path, **kw):
    kw.setdefault("lease_duration", 0.6)
    kw.setdefault("renew_deadline", 0.4)
    kw.setdefault("retry_period", 0.05)
    return LeaseElector(str(path), **kw)


def test_single_holder_and_release_handover(tmp_path):
    lease = tmp_path / "epp.lease"
    a, b = _mk(lease, identity="a"), _mk(lease, identity="b")
    a.tick()
    b.tick()
    assert a.is_leader and not b.is_leader and a.holder() == "a"
    for _ in range(5):  # renewals keep it
        a.tick()
        b.tick()
    assert a.is_leader and not b.is_leader
    a.stop()            # clean shutdown releases: b takes over at once
    b.tick()
    assert b.is_leader and b.holder() == "b"


def test_dead_holder_expires_and_stalled_leader_steps_down(tmp_path):
    lease = tmp_path / "epp.lease"
    events = []
    a = _mk(lease, identity="a", on_stopped_leading=lambda: events.append("a-stop"))
    b = _mk(lease, identity="b", on_started_leading=lambda: events.append("b-start"))
    a.tick()
    assert a.is_leader
    b.tick()
    assert not b.is_leader          # lease still valid
    time.sleep(0.7)                 # a stalls past its lease duration
    b.tick()
    assert b.is_leader and events == ["b-start"]
    a.tick()                        # a wakes up: the lease is b's, a must not act
    assert not a.is_leader and "a-stop" in events
    with pytest.raises(ValueError):
        LeaseElector(str(lease), lease_duration=1, renew_deadline=2, retry_period=0.1)


def test_concurrent_candidates_never_share(tmp_path):
    lease = tmp_path / "epp.lease"
    es = [_mk(lease, identity=f"c{i}") for i in range(6)]
    for _ in range(20):
        for e in es:
            e.tick()
        assert sum(e.is_leader for e in es) == 1


def test_wva_standby_does_not_actuate(tmp_path):
    from llmd_amd.autoscale.wva import Variant, WVAEngine

    class Act:
        def __init__(self):
            self.calls = 0

        def scale(self, v, n):
            self.calls += 1

    lease = tmp_path / "wva.lease"
    lead, stand = _mk(lease, identity="w1"), _mk(lease, identity="w2")
    lead.tick()
    stand.tick()
    acts = [Act(), Act()]
    engines = [WVAEngine({}, actuator=acts[0], elector=lead), WVAEngine({}, actuator=acts[1], elector=stand)]
    for eng in engines:
        pools = {"m": [Variant(name="v", model_id="m", current=1, min_replicas=1, max_replicas=4, cost=1.0)]}
        eng.step(pools)
    assert acts[0].calls > 0 and acts[1].calls == 0


def _start_router(port, lease, sim_port):
    cmd = [sys.executable, "-m", "llmd_amd.router.proxy", "--port", str(port), "--metrics-port", "0",
           "--endpoints", f"127.0.0.1:{sim_port}", "--ha-enable-leader-election", "--ha-lease-file", str(lease),
           "--ha-lease-duration", "1.5", "--ha-renew-deadline", "1.0", "--ha-retry-period", "0.2"]
    return subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            start_new_session=True)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_router_ha_failover_over_http(tmp_path):
    """Two router replicas share a lease: exactly one reports ready and serves;
    killing it (no release) hands traffic to the standby within the lease."""
    from llmd_amd.sim.server import start_sim

    async def main():
        runner, _, sim_port = await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001)
        lease = tmp_path / "epp.lease"
        ports = [_free_port(), _free_port()]
        procs = [_start_router(p, lease, sim_port) for p in ports]
        try:
            async with aiohttp.ClientSession() as s:
                async def status(p):
                    try:
                        async with s.get(f"http://127.0.0.1:{p}/health") as r:
                            return r.status
                    except aiohttp.ClientError:
                        return None

                deadline = time.time() + 60
                while time.time() < deadline:
                    st = [await status(p) for p in ports]
                    if sorted(x or 0 for x in st) == [200, 503]:
                        break
                    await asyncio.sleep(0.2)
                assert sorted(x or 0 for x in st) == [200, 503], st
                li = st.index(200)
                body = {"model": "m", "prompt": "hello", "max_tokens": 2}
                async with s.post(f"http://127.0.0.1:{ports[li]}/v1/completions", json=body) as r:
                    assert r.status == 200
                async with s.post(f"http://127.0.0.1:{ports[1 - li]}/v1/completions", json=body) as r:
                    assert r.status == 503 and r.headers.get("x-llm-d-epp-role") == "standby"
                os.killpg(procs[li].pid, 9)   # leader dies without releasing
                procs[li].wait()
                deadline = time.time() + 20
                while time.time() < deadline and await status(ports[1 - li]) != 200:
                    await asyncio.sleep(0.2)
                assert await status(ports[1 - li]) == 200
                async with s.post(f"http://127.0.0.1:{ports[1 - li]}/v1/completions", json=body) as r:
                    assert r.status == 200
        finally:
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, 9)
                    p.wait()
            await runner.cleanup()

    asyncio.run(main())
