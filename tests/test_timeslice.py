"""RL time-slicing (llmd_amd/rl/timeslice.py; SURVEY C43,
proposals/rl-time-slicing-platform.md): exclusive GPU phases, warm grants,
eviction of the resident job, a dead job's forced eviction, duty cycle of two
interleaved jobs vs. one, the trainer tensor swapper (CPU round trip; GPU
memory release and host-link bandwidth) and the engine swapper against the
real API server."""
import asyncio
import socket
import threading
import time
import urllib.request

import pytest
import torch
from aiohttp import web

from llmd_amd.rl.timeslice import EngineSwapper, Orchestrator, Slicer, TensorSwapper


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Server:
    """An aiohttp app on its own loop thread."""

    def __init__(self, make_app):
        self.port = _free_port()
        self.loop = asyncio.new_event_loop()
        self.obj = None
        ready = threading.Event()

        def run():
            asyncio.set_event_loop(self.loop)

            async def start():
                self.obj, app = make_app()
                self.runner = web.AppRunner(app)
                await self.runner.setup()
                await web.TCPSite(self.runner, "127.0.0.1", self.port).start()
                ready.set()
            self.loop.run_until_complete(start())
            self.loop.run_forever()

        self.thread = threading.Thread(target=run, daemon=True)
        self.thread.start()
        assert ready.wait(30)
        self.url = f"http://127.0.0.1:{self.port}"

    def stop(self):
        asyncio.run_coroutine_threadsafe(self.runner.cleanup(), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(10)


def _orch(evict_timeout=5.0):
    def make():
        o = Orchestrator(evict_timeout)
        return o, o.app()
    return _Server(make)


def test_exclusive_phases_warm_grants_and_eviction():
    srv = _orch()
    log, lock = [], threading.Lock()
    active = []

    def swapper(job, what):
        def f():
            with lock:
                log.append((job, what))
        return f

    try:
        a = Slicer("a", srv.url, kind="trainer", swap_in=swapper("a", "in"), swap_out=swapper("a", "out"))
        b = Slicer("b", srv.url, kind="sampler", swap_in=swapper("b", "in"), swap_out=swapper("b", "out"))

        @a.run_on_gpu
        def phase_a():
            active.append("a")
            assert active.count("a") == 1 and "b" not in active
            time.sleep(0.02)
            active.remove("a")

        # one job alone: cold first grant, warm afterwards, no swaps
        phase_a()
        phase_a()
        assert log == [("a", "in")]
        st = srv.obj.status()
        assert st["jobs"]["a"]["grants"] == 2 and st["jobs"]["a"]["warm_grants"] == 1
        # b needs the GPUs: the resident a swaps out before b swaps in
        with b.gpu() as g:
            assert not g["warm"]
            assert log[-2:] == [("a", "out"), ("b", "in")]
        # interleave both from threads: never two phases at once
        def loop_b():
            for _ in range(5):
                with b.gpu():
                    active.append("b")
                    assert "a" not in active
                    time.sleep(0.02)
                    active.remove("b")
                time.sleep(0.01)
        t = threading.Thread(target=loop_b)
        t.start()
        for _ in range(5):
            phase_a()
            time.sleep(0.01)
        t.join(30)
        assert not t.is_alive()
        outs = [x for x in log if x[1] == "out"]
        ins = [x for x in log if x[1] == "in"]
        assert len(ins) - len(outs) == 1  # exactly one job resident at the end
        text = urllib.request.urlopen(srv.url + "/metrics", timeout=5).read().decode()
        assert 'timeslice_grants_total{job="a",kind="trainer",warm="true"}' in text
        assert "timeslice_swap_out_seconds_count" in text
        a.close()
        b.close()
    finally:
        srv.stop()


def test_dead_resident_job_is_force_evicted():
    srv = _orch(evict_timeout=0.5)
    try:
        a = Slicer("a", srv.url)
        with a.gpu():
            pass
        a.close()  # the job "dies": its evict thread stops answering
        time.sleep(2.5)
        b = Slicer("b", srv.url)
        t = time.time()
        with b.gpu():
            pass
        assert time.time() - t < 5
        assert srv.obj.forced_evictions == 1
        b.close()
    finally:
        srv.stop()


def test_interleaving_raises_duty_cycle():
    """Two jobs that are each 1/3 on the GPU and 2/3 blocked: alone the pool
    is busy ~1/3 of the time, interleaved roughly twice that."""
    def run(n_jobs):
        srv = _orch()
        try:
            slicers = [Slicer(f"j{i}", srv.url) for i in range(n_jobs)]

            def job(s):
                for _ in range(6):
                    with s.gpu():
                        time.sleep(0.05)
                    time.sleep(0.1)  # reward computation on the CPU
            ts = [threading.Thread(target=job, args=(s,)) for s in slicers]
            t0 = time.time()
            for t in ts:
                t.start()
            for t in ts:
                t.join(60)
            wall = time.time() - t0
            duty = srv.obj.duty_cycle()
            for s in slicers:
                s.close()
            return duty, wall
        finally:
            srv.stop()

    d1, w1 = run(1)
    d2, w2 = run(2)
    assert d2 > 1.4 * d1, (d1, d2)
    assert w2 < 1.7 * w1, (w1, w2)  # two jobs finish in far less than twice the time


def _model_and_opt(device):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 8)).to(device)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2)
    x = torch.randn(32, 64, device=device)
    for _ in range(2):
        opt.zero_grad()
        m(x).square().mean().backward()
        opt.step()
    return m, opt, x


def test_tensor_swapper_round_trip_cpu():
    m, opt, x = _model_and_opt("cpu")
    ref_m, ref_opt, _ = _model_and_opt("cpu")
    sw = TensorSwapper(m, opt)
    for _ in range(2):  # second round trip takes the packed (one copy per dtype) path
        sw.swap_out()
        assert all(p.numel() == 0 for p in m.parameters())
        sw.swap_in()
    for p, q in zip(m.parameters(), ref_m.parameters()):
        assert torch.equal(p, q) and torch.equal(p.grad, q.grad)
    # training continues identically after the swaps
    for mm, oo in ((m, opt), (ref_m, ref_opt)):
        oo.zero_grad()
        mm(x).square().mean().backward()
        oo.step()
    for p, q in zip(m.parameters(), ref_m.parameters()):
        assert torch.equal(p, q)


@pytest.mark.gpu
def test_tensor_swapper_gpu_memory_and_bandwidth():
    dev = torch.device("cuda:0")
    big = [torch.randn(256 * 1024 * 1024 // 2, device=dev, dtype=torch.bfloat16) for _ in range(8)]  # 2 GiB
    keep = [t.clone() for t in big[:1]]
    sw = TensorSwapper(tensors=big)
    sw.swap_out()
    sw.swap_in()  # tensors now view one buffer: the next round trip is one copy each way
    torch.cuda.synchronize()
    before = torch.cuda.memory_allocated(dev)
    t = time.perf_counter()
    sw.swap_out()
    t_out = time.perf_counter() - t
    after = torch.cuda.memory_allocated(dev)
    assert before - after >= sw.bytes * 0.99
    t = time.perf_counter()
    sw.swap_in()
    t_in = time.perf_counter() - t
    assert torch.equal(big[0], keep[0])
    gbps_out, gbps_in = sw.bytes / t_out / 1e9, sw.bytes / t_in / 1e9
    print(f"trainer swap {sw.bytes / 2**30:.1f} GiB: out {t_out * 1e3:.0f} ms ({gbps_out:.1f} GB/s), "
          f"in {t_in * 1e3:.0f} ms ({gbps_in:.1f} GB/s)")
    assert gbps_out > 5 and gbps_in > 5


def test_engine_swapper_against_api_server():
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.serving.api_server import build_server

    def make():
        cfg = EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                                  max_num_batched_tokens=128, max_num_seqs=4, max_model_len=512,
                                  enforce_eager=True)
        s = build_server(cfg)
        return s, s.app()
    srv = _Server(make)
    try:
        orch = _orch()
        sw = EngineSwapper(srv.url, level=1)
        s = Slicer("sampler", orch.url, swap_in=sw.swap_in, swap_out=sw.swap_out)
        other = Slicer("trainer", orch.url)
        with s.gpu():
            pass
        with other.gpu():  # evicts the sampler: the engine sleeps
            import json
            st = json.loads(urllib.request.urlopen(srv.url + "/is_sleeping", timeout=5).read())
            assert st["is_sleeping"] and st["level"] == 1
        with s.gpu():
            st = json.loads(urllib.request.urlopen(srv.url + "/is_sleeping", timeout=5).read())
            assert not st["is_sleeping"]
        s.close()
        other.close()
        orch.stop()
    finally:
        srv.stop()
        srv.obj.aeng.shutdown()
