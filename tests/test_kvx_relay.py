"""kvx multi-link striping (kvx/agent.py, the UCCL multi-path role): a large
pull is split over the direct link and two-hop paths through relay agents.

CPU: the split plan. GPU (one device, three processes - prefiller P, relay R,
decoder D - sharing cuda:0 through hipIpc, as the symm tests do): D pulls a
request's blocks with R as relay and gets P's bytes exactly, for a TP-equal
pull and for a decoder holding half of P's KV heads."""
import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

from llmd_amd.kvx.agent import stripe_plan

L, NB, PL, H, BS, D = 4, 64, 2, 8, 16, 64


def test_stripe_plan_covers_every_block_once():
    for n in (1, 2, 7, 64, 1000):
        for k in (0, 1, 3, 6):
            plan = stripe_plan(n, k)
            assert len(plan) == 1 + k
            covered = [i for a, b in plan for i in range(a, b)]
            assert covered == list(range(n))
            sizes = [b - a for a, b in plan]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pool(seed, heads=H):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(L, NB, PL, heads, BS, D, generator=g).to(torch.bfloat16)


def _proc(role, q_out, q_in, heads, dev=0):
    os.environ["LLMD_KVX_HEARTBEAT_S"] = "0"
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(dev)
    from llmd_amd.kvx import agent as A

    try:
        if role == "P":
            ag = A.KvxAgent(_pool(1).cuda(), transport="ipc")
            prm = ag.hold("r", 1, list(range(5, 45)), 40 * BS)
            q_out.put(("P", prm))
            q_in.get()  # until the decoder is done
            ag.close()
        elif role == "R":
            ag = A.KvxAgent(torch.zeros(L, NB, PL, H, BS, D, dtype=torch.bfloat16, device="cuda"),
                            transport="ipc")
            q_out.put(("R", (ag.host, ag.port)))
            q_in.get()
            ag.close()
        else:
            prm, relay = q_in.get()
            kv = torch.zeros(L, NB, PL, heads, BS, D, dtype=torch.bfloat16, device="cuda")
            ag = A.KvxAgent(kv, transport="ipc", exports=False, relays=[relay], stripe_min_bytes=1,
                            tp_rank=0 if heads == H else 1, tp_size=H // heads)
            local = list(range(20, 60))
            ag.start_load("r", prm, local)
            done = []
            t = time.monotonic() + 60
            while not done and time.monotonic() < t:
                done = ag.poll_done() if ag.tp_size == 1 else list(ag.done.queue) or (
                    [("r", ag.tp_wait["r"][1])] if ag.tp_wait.get("r", [0])[0] >= 1 else [])
                time.sleep(0.01)
            src = _pool(1)
            h0 = 0 if heads == H else heads
            got = kv.cpu()[:, local]
            want = src[:, prm["remote_block_ids"], :, h0:h0 + heads]
            q_out.put(("D", {"done": done, "bad": int((got != want).sum()),
                             "relay_maps": sum(1 for k in ag.ipc_maps if str(k).startswith("relay:"))}))
            ag.close()
    except Exception as e:  # noqa: BLE001
        q_out.put((role, f"error: {e!r}"))


NGPU = torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("devices", [(0, 0, 0), pytest.param((0, 1, 2), marks=pytest.mark.skipif(
    NGPU < 3, reason="needs 3 GPUs: P, relay and D on their own devices (two-hop xGMI path)"))])
@pytest.mark.parametrize("heads", [H, H // 2])
def test_striped_pull_through_relay(heads, devices):
    ctx = mp.get_context("spawn")
    q_out, qp, qr, qd = ctx.Queue(), ctx.Queue(), ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_proc, args=(r, q_out, qi, heads, d))
             for (r, qi), d in zip((("P", qp), ("R", qr), ("D", qd)), devices)]
    for p in procs:
        p.start()
    try:
        got = {}
        while len(got) < 2:
            role, val = q_out.get(timeout=120)
            assert not (isinstance(val, str) and val.startswith("error")), (role, val)
            got[role] = val
        qd.put((got["P"], got["R"]))
        role, res = q_out.get(timeout=120)
        assert role == "D" and isinstance(res, dict), (role, res)
        assert res["done"] == [("r", True)], res
        assert res["bad"] == 0, res
        assert res["relay_maps"] == 1  # the relay path really ran (its staging was mapped)
    finally:
        qp.put(1)
        qr.put(1)
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
