"""Collaborative GPU time-slicing for RL jobs (the design of
proposals/rl-time-slicing-platform.md:15-62).

RL loops leave the accelerators idle during their blocking phases (reward
evaluation on the CPU, stragglers, synchronisation). Several jobs can share
one node if each yields the GPUs while it blocks and the swap is fast:

* a local **orchestrator** (this module's HTTP daemon) owns the GPU lease of
  a pool and queues the jobs that want it (FIFO within a priority);
* a job marks its GPU phases with ``@slicer.run_on_gpu`` (or ``with
  slicer.gpu():``). Entering a phase waits for the lease; leaving it releases
  the lease but keeps the job's context **resident** until another job
  actually needs the GPUs - a job that re-enters with nobody in between gets
  a warm grant and swaps nothing;
* when another job is granted, the orchestrator asks the resident job to
  swap out (its client's evict thread) and waits for the ack (or for
  ``evictTimeout``: a dead job's memory is already gone);
* swappers: ``EngineSwapper`` for a sampler (this repo's API server: ``POST
  /sleep`` level 2 drops the weights and the KV pool - the trainer re-pushes
  weights each step anyway - or level 1 keeps the weights in pinned host
  memory; ``/wake_up`` returns), ``TensorSwapper`` for a trainer (parameters,
  gradients and optimizer state packed per dtype into one pinned host arena;
  after the first round trip the tensors are views of one device buffer per
  dtype, so a swap is ONE D2H / H2D copy per dtype at host-link bandwidth
  instead of one launch per tensor).

``/metrics`` exports the pool duty cycle (fraction of wall time a job held the
GPUs), per-job GPU seconds, grants (warm / cold), swaps and swap-out latency -
the proposal's duty-cycle and warm-swap numbers.

  python -m llmd_amd.rl.timeslice --port 8490
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import threading
import time
import urllib.error
import urllib.request
from collections import defaultdict
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import Callable, Optional

from aiohttp import web

log = logging.getLogger("llmd.timeslice")


# ------------------------------------------------------------------ orchestrator
@dataclass
class _Job:
    name: str
    kind: str = "sampler"
    priority: int = 0
    gpu_s: float = 0.0
    grants: int = 0
    warm_grants: int = 0
    swaps_out: int = 0
    evict: asyncio.Event = field(default_factory=asyncio.Event)
    evicted: asyncio.Event = field(default_factory=asyncio.Event)


class Orchestrator:
    """One GPU pool's lease. All state lives on the event loop (no locks)."""

    def __init__(self, evict_timeout: float = 30.0):
        self.evict_timeout = evict_timeout
        self.jobs: dict[str, _Job] = {}
        self.holder: Optional[str] = None
        self.resident: Optional[str] = None
        self.waiting: list[tuple[int, int, str, asyncio.Future]] = []  # (-prio, seq, job, fut)
        self._seq = 0
        self._t0: Optional[float] = None
        self._held_since: Optional[float] = None
        self.busy_s = 0.0
        self.swap_s: list[float] = []
        self.forced_evictions = 0
        self._granting = False

    def register(self, name: str, kind: str = "sampler", priority: int = 0) -> _Job:
        j = self.jobs.get(name)
        if j is None:
            j = self.jobs[name] = _Job(name, kind, priority)
        j.kind, j.priority = kind, priority
        return j

    async def acquire(self, name: str) -> dict:
        j = self.jobs.get(name) or self.register(name)
        if self.holder == name:
            raise RuntimeError(f"job {name} already holds the GPUs")
        fut = asyncio.get_running_loop().create_future()
        self._seq += 1
        self.waiting.append((-j.priority, self._seq, name, fut))
        self.waiting.sort(key=lambda w: w[:2])
        asyncio.get_running_loop().create_task(self._grant_next())
        try:
            return await fut
        except asyncio.CancelledError:  # client went away while waiting
            self.waiting = [w for w in self.waiting if w[3] is not fut]
            if fut.done() and not fut.cancelled() and self.holder == name:
                self.release(name)
            raise

    async def _grant_next(self):
        if self._granting or self.holder is not None or not self.waiting:
            return
        self._granting = True
        try:
            _, _, name, fut = self.waiting.pop(0)
            warm = self.resident == name
            if self.resident is not None and not warm:
                await self._evict(self.resident)
            if fut.cancelled():
                return
            now = time.monotonic()
            if self._t0 is None:
                self._t0 = now
            self.holder, self.resident, self._held_since = name, name, now
            j = self.jobs[name]
            j.grants += 1
            j.warm_grants += int(warm)
            fut.set_result({"granted": True, "warm": warm})
        finally:
            self._granting = False
            if self.holder is None and self.waiting:
                asyncio.get_running_loop().create_task(self._grant_next())

    async def _evict(self, name: str):
        j = self.jobs[name]
        j.evicted.clear()
        j.evict.set()
        t = time.monotonic()
        try:
            await asyncio.wait_for(j.evicted.wait(), self.evict_timeout)
            self.swap_s.append(time.monotonic() - t)
        except asyncio.TimeoutError:
            log.warning("job %s did not swap out within %.0fs: taking the GPUs anyway", name, self.evict_timeout)
            self.forced_evictions += 1
        j.evict.clear()
        self.resident = None

    def release(self, name: str, yield_now: bool = False):
        if self.holder != name:
            raise RuntimeError(f"job {name} does not hold the GPUs (holder {self.holder})")
        now = time.monotonic()
        self.busy_s += now - self._held_since
        self.jobs[name].gpu_s += now - self._held_since
        self.holder = None
        if yield_now:  # the job swapped out eagerly (it knows its next blocking phase is long)
            self.resident = None
        asyncio.get_running_loop().create_task(self._grant_next())

    async def wait_evict(self, name: str, timeout: float) -> bool:
        j = self.jobs.get(name) or self.register(name)
        try:
            await asyncio.wait_for(j.evict.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    def ack_evicted(self, name: str):
        j = self.jobs.get(name)
        if j is not None:
            j.swaps_out += 1
            j.evicted.set()

    def duty_cycle(self) -> float:
        if self._t0 is None:
            return 0.0
        busy = self.busy_s + (time.monotonic() - self._held_since if self.holder else 0.0)
        return busy / max(1e-9, time.monotonic() - self._t0)

    def status(self) -> dict:
        return {"holder": self.holder, "resident": self.resident, "waiting": [w[2] for w in self.waiting],
                "duty_cycle": self.duty_cycle(), "forced_evictions": self.forced_evictions,
                "jobs": {n: {"kind": j.kind, "priority": j.priority, "gpu_s": j.gpu_s, "grants": j.grants,
                             "warm_grants": j.warm_grants, "swaps_out": j.swaps_out} for n, j in self.jobs.items()}}

    def render_metrics(self) -> str:
        out = ["# TYPE timeslice_duty_cycle gauge", f"timeslice_duty_cycle {self.duty_cycle():.6f}",
               "# TYPE timeslice_queue_length gauge", f"timeslice_queue_length {len(self.waiting)}",
               "# TYPE timeslice_forced_evictions_total counter",
               f"timeslice_forced_evictions_total {self.forced_evictions}",
               "# TYPE timeslice_job_gpu_seconds_total counter", "# TYPE timeslice_grants_total counter",
               "# TYPE timeslice_swaps_out_total counter"]
        for n, j in sorted(self.jobs.items()):
            lab = f'job="{n}",kind="{j.kind}"'
            out += [f"timeslice_job_gpu_seconds_total{{{lab}}} {j.gpu_s:.6f}",
                    f'timeslice_grants_total{{{lab},warm="true"}} {j.warm_grants}',
                    f'timeslice_grants_total{{{lab},warm="false"}} {j.grants - j.warm_grants}',
                    f"timeslice_swaps_out_total{{{lab}}} {j.swaps_out}"]
        if self.swap_s:
            s = sorted(self.swap_s)
            out += ["# TYPE timeslice_swap_out_seconds summary",
                    f'timeslice_swap_out_seconds{{quantile="0.5"}} {s[len(s) // 2]:.6f}',
                    f'timeslice_swap_out_seconds{{quantile="1"}} {s[-1]:.6f}',
                    f"timeslice_swap_out_seconds_count {len(s)}"]
        return "\n".join(out) + "\n"

    def app(self) -> web.Application:
        app = web.Application()

        async def register(req):
            b = await req.json()
            self.register(b["job"], b.get("kind", "sampler"), int(b.get("priority", 0)))
            return web.json_response({"ok": True})

        async def acquire(req):
            b = await req.json()
            try:
                return web.json_response(await self.acquire(b["job"]))
            except RuntimeError as e:
                return web.json_response({"error": str(e)}, status=409)

        async def release(req):
            b = await req.json()
            try:
                self.release(b["job"], bool(b.get("yield_now", False)))
            except RuntimeError as e:
                return web.json_response({"error": str(e)}, status=409)
            return web.json_response({"ok": True})

        async def evict(req):
            ev = await self.wait_evict(req.query["job"], float(req.query.get("timeout", 20)))
            return web.json_response({"evict": ev})

        async def evicted(req):
            self.ack_evicted((await req.json())["job"])
            return web.json_response({"ok": True})

        async def status(_):
            return web.json_response(self.status())

        async def metrics(_):
            return web.Response(text=self.render_metrics(), content_type="text/plain")

        async def healthz(_):
            return web.Response(text="ok")

        r = app.router
        r.add_post("/register", register)
        r.add_post("/acquire", acquire)
        r.add_post("/release", release)
        r.add_get("/evict", evict)
        r.add_post("/evicted", evicted)
        r.add_get("/status", status)
        r.add_get("/metrics", metrics)
        r.add_get("/healthz", healthz)
        return app


# ------------------------------------------------------------------ client
def _post(url: str, body: dict, timeout: Optional[float] = None) -> dict:
    req = urllib.request.Request(url, data=json.dumps(body).encode(), headers={"content-type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read())


class Slicer:
    """A job's handle on the orchestrator. ``swap_in`` / ``swap_out`` move the
    job's GPU context; they never run concurrently with each other or with a
    GPU phase of this job."""

    def __init__(self, job: str, url: str, kind: str = "sampler", priority: int = 0,
                 swap_in: Optional[Callable[[], None]] = None, swap_out: Optional[Callable[[], None]] = None):
        self.job, self.url = job, url.rstrip("/")
        self.swap_in_fn, self.swap_out_fn = swap_in, swap_out
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.resident = False
        self.swap_in_s: list[float] = []
        self.swap_out_s: list[float] = []
        self.last_phase_s = 0.0
        _post(self.url + "/register", {"job": job, "kind": kind, "priority": priority})
        self._evict_thread = threading.Thread(target=self._evict_loop, daemon=True, name=f"slicer-{job}")
        self._evict_thread.start()

    def _evict_loop(self):
        while not self._stop.is_set():
            try:
                with urllib.request.urlopen(f"{self.url}/evict?job={self.job}&timeout=2", timeout=10) as r:
                    ev = json.loads(r.read()).get("evict")
            except (OSError, urllib.error.URLError, ValueError):
                if self._stop.wait(0.2):
                    return
                continue
            if ev:
                with self._lock:
                    self._swap_out()
                try:
                    _post(self.url + "/evicted", {"job": self.job}, timeout=10)
                except OSError:
                    pass

    def _swap_out(self):
        if self.resident and self.swap_out_fn is not None:
            t = time.perf_counter()
            self.swap_out_fn()
            self.swap_out_s.append(time.perf_counter() - t)
        self.resident = False

    @contextmanager
    def gpu(self, yield_after: bool = False):
        """A GPU phase. ``yield_after``: swap out right away on exit (the job
        knows its next blocking phase is long) instead of staying resident."""
        try:
            g = _post(self.url + "/acquire", {"job": self.job})
        except OSError:
            # the grant may have happened with the reply lost: hand it back
            try:
                _post(self.url + "/release", {"job": self.job}, timeout=10)
            except OSError:
                pass
            raise
        with self._lock:
            if not (g["warm"] and self.resident):
                if self.swap_in_fn is not None:
                    t = time.perf_counter()
                    self.swap_in_fn()
                    self.swap_in_s.append(time.perf_counter() - t)
                self.resident = True
            t0 = time.perf_counter()
            try:
                yield g
            finally:
                if yield_after:
                    self._swap_out()
                self.last_phase_s = time.perf_counter() - t0
                _post(self.url + "/release", {"job": self.job, "yield_now": yield_after}, timeout=30)

    def run_on_gpu(self, fn):
        """Decorator form of :meth:`gpu` (the proposal's ``@slicer.run_on_gpu``)."""
        def wrapped(*a, **kw):
            with self.gpu():
                return fn(*a, **kw)
        wrapped.__name__ = getattr(fn, "__name__", "gpu_phase")
        return wrapped

    def close(self):
        self._stop.set()


# ------------------------------------------------------------------ swappers
class EngineSwapper:
    """Sampler context = an engine served by this repo's API server."""

    def __init__(self, url: str, level: int = 2, timeout: float = 120.0):
        self.url, self.level, self.timeout = url.rstrip("/"), level, timeout

    def swap_out(self):
        _post(self.url + "/sleep", {"level": self.level}, timeout=self.timeout)

    def swap_in(self):
        _post(self.url + "/wake_up", {}, timeout=self.timeout)


class TensorSwapper:
    """Trainer context = a set of device tensors (module parameters and their
    gradients, optimizer state). ``swap_out`` copies them per dtype into one
    pinned host arena (allocated once) and frees the device memory;
    ``swap_in`` allocates ONE device buffer per dtype, copies the arena in with
    a single H2D and re-points every tensor at its slice, so later swap-outs
    are one D2H per dtype too."""

    def __init__(self, module=None, optimizer=None, tensors: Optional[list] = None):
        import torch

        self.torch = torch
        self.module, self.optimizer = module, optimizer
        self.extra = list(tensors or [])
        self.arenas: dict = {}      # dtype -> host tensor (pinned for a GPU context)
        self.layout: list = []      # (tensor, dtype, offset, numel, shape)
        self._bufs: dict = {}       # dtype -> device buffer the tensors view (after swap_in)
        self.device = None
        self.on_device = True
        self.bytes = 0

    def _tensors(self) -> list:
        ts = []
        if self.module is not None:
            for p in self.module.parameters():
                ts.append(p)
                if p.grad is not None:
                    ts.append(p.grad)
        if self.optimizer is not None:
            for st in self.optimizer.state.values():
                ts += [v for v in st.values() if self.torch.is_tensor(v) and v.numel() > 1]
        seen, out = set(), []
        for t in ts + self.extra:
            if id(t) not in seen:
                seen.add(id(t))
                out.append(t)
        return out

    def _packed(self, dt) -> bool:
        b = self._bufs.get(dt)
        if b is None:
            return False
        base, es = b.data_ptr(), b.element_size()
        return all(t.numel() == nm and t.data_ptr() == base + off * es
                   for t, d, off, nm, _ in self.layout if d == dt)

    def swap_out(self):
        torch = self.torch
        if not self.on_device:
            return
        ts = self._tensors()
        if not ts:
            self.on_device = False
            return
        self.device = ts[0].device
        pin = self.device.type == "cuda"
        if [t for t, *_ in self.layout] != ts:  # first swap, or the tensor set changed
            by_dtype: dict = defaultdict(list)
            for t in ts:
                by_dtype[t.dtype].append(t)
            self.layout, self._bufs = [], {}
            for dt, group in by_dtype.items():
                n = sum(t.numel() for t in group)
                a = self.arenas.get(dt)
                if a is None or a.numel() < n:
                    self.arenas[dt] = torch.empty(n, dtype=dt, pin_memory=pin)
                off = 0
                for t in group:
                    self.layout.append((t, dt, off, t.numel(), tuple(t.shape)))
                    off += t.numel()
        self.bytes = sum(nm * t.element_size() for t, _, _, nm, _ in self.layout)
        for dt in {d for _, d, _, _, _ in self.layout}:
            if self._packed(dt):
                b = self._bufs[dt]
                self.arenas[dt][:b.numel()].copy_(b, non_blocking=pin)
            else:
                for t, d, off, nm, _ in self.layout:
                    if d == dt:
                        self.arenas[dt][off:off + nm].copy_(t.detach().reshape(-1), non_blocking=pin)
        if pin:
            torch.cuda.current_stream(self.device).synchronize()
        for t, dt, _, _, _ in self.layout:
            t.data = torch.empty(0, dtype=dt, device=self.device)
        self._bufs = {}
        if pin:
            torch.cuda.empty_cache()  # hand the memory back for the other job's process
        self.on_device = False

    def swap_in(self):
        torch = self.torch
        if self.on_device:
            return
        pin = self.device is not None and self.device.type == "cuda"
        bufs = {}
        for dt, a in self.arenas.items():
            n = sum(nm for _, d, _, nm, _ in self.layout if d == dt)
            b = torch.empty(n, dtype=dt, device=self.device)
            b.copy_(a[:n], non_blocking=pin)
            bufs[dt] = b
        for t, dt, off, nm, shape in self.layout:
            t.data = bufs[dt][off:off + nm].view(shape)
        self._bufs = bufs
        if pin:
            torch.cuda.current_stream(self.device).synchronize()
        self.on_device = True


# ------------------------------------------------------------------ CLI
def serve(port: int, evict_timeout: float = 30.0, host: str = "127.0.0.1"):
    async def _run():
        orch = Orchestrator(evict_timeout)
        runner = web.AppRunner(orch.app())
        await runner.setup()
        await web.TCPSite(runner, host, port).start()
        log.info("time-slice orchestrator on %s:%d", host, port)
        await asyncio.Event().wait()

    asyncio.run(_run())


def main(argv=None):
    p = argparse.ArgumentParser("llmd-amd RL time-slice orchestrator")
    p.add_argument("--port", type=int, default=8490)
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--evict-timeout", type=float, default=30.0)
    p.add_argument("--log-level", default="info")
    a = p.parse_args(argv)
    logging.basicConfig(level=a.log_level.upper(), format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    serve(a.port, a.evict_timeout, a.host)


if __name__ == "__main__":
    main()
