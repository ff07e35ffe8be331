"""P/D-disaggregated serving benchmark driver (used by bench.py --mode pd).

Topology inside one torchrun job (one process per GPU):
  ranks [0, P)   prefill engines, each serving the real OpenAI endpoint on
                 127.0.0.1:<base+rank> (AsyncEngine + aiohttp) with a
                 ``kv_transfer_config`` (kvx producer);
  ranks [P, N)   decode engines (kvx consumer, IPC pull over xGMI), in
                 groups of ``--decode-tp`` consecutive ranks (one TP replica
                 each: the reference's P/D headline runs its decoders TP4,
                 guides/pd-disaggregation/README.md:336-460). The group's
                 first rank is the TP driver (scheduler + sidecar), the
                 others TP followers (engine/tp_worker.py) that pull their
                 own KV-head slice. The driver is driven by
                 an in-process routing-sidecar loop: every new request is sent
                 to a prefill rank (least outstanding) with
                 ``kv_transfer_params{do_remote_decode}`` / ``max_tokens=1``,
                 the returned params are handed to the local decoder which
                 pulls the KV and decodes (the reference's nixlv2 protocol,
                 docs/architecture/advanced/disaggregation/README.md:119-131).
Why TP on the decode side: a decode GPU is KV-capacity bound. A TP1 70B
replica spends 141 GB of HBM on weights and fits ~64 ISL-5000 sequences
(50.9 ms/step -> ~1260 tok/s per GPU); a TP2 replica holds half the weights
per GPU, so the same two GPUs fit ~3x the sequences and read each weight byte
once per step for twice the rows.
Timing: K decode steps on every decode driver between gloo barriers (+ device
sync); prefill ranks serve continuously. Reported value = total output
tokens / max elapsed; TTFT measured at the decode side from the moment the
prefill request is issued (the "true TTFT" a client would see).
"""
from __future__ import annotations

import asyncio
import datetime
import json
import os
import queue
import statistics
import sys
import threading
import time

import numpy as np
import torch
import torch.distributed as dist


def _sync(a):
    if a.device == "cuda":
        torch.cuda.synchronize()


def run_pd(a, rank: int, world: int, local_rank: int, log) -> dict | None:
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    def log(_rank, *m):  # every rank reports (hang diagnosis on multi-GPU runs)
        print(f"[bench-pd rank {rank}]", *m, file=sys.stderr, flush=True)

    P = a.prefill_gpus or max(1, (3 * world) // 4)
    if not 0 < P < world:
        raise SystemExit(f"pd mode needs 0 < prefill ranks ({P}) < world ({world})")
    n_dec = world - P
    dtp = a.decode_tp or (2 if n_dec % 2 == 0 else 1)
    if n_dec % dtp:
        raise SystemExit(f"pd mode: {n_dec} decode ranks not divisible by --decode-tp {dtp}")
    is_prefill = rank < P
    # explicit timeouts: a cross-device failure must end the job with an error, not hang it
    to = datetime.timedelta(seconds=int(os.environ.get("LLMD_DIST_TIMEOUT", "1800")))
    world_ctl = dist.new_group(backend="gloo", timeout=to)
    drivers = list(range(P, world, dtp))
    # timing / result group: prefill ranks + decode drivers (followers sit in
    # their step-plan loop and are released by the driver's shutdown)
    ctl = dist.new_group(list(range(P)) + drivers, backend="gloo", timeout=to) if dtp > 1 else world_ctl
    is_follower = False
    if dtp > 1:
        from llmd_amd.parallel.state import ParallelState, set_state

        for d in drivers:  # collective: every rank creates every group
            ranks = list(range(d, d + dtp))
            tg = dist.new_group(ranks, timeout=to)
            tgc = dist.new_group(ranks, backend="gloo", timeout=to)
            if rank in ranks:
                set_state(ParallelState(world_size=world, rank=rank, local_rank=local_rank, tp_size=dtp,
                                        tp_rank=rank - d, tp_group=tg, tp_cpu_group=tgc, cpu_group=tgc,
                                        backend=dist.get_backend(), tp_src=d))
                is_follower = rank != d
    if os.environ.get("LLMD_KVX_TRANSPORT", "auto") == "rccl":
        # two-sided RCCL send/recv KV transport: a group used by kvx only (collective creation)
        from llmd_amd.kvx.agent import set_p2p_group

        set_p2p_group(dist.new_group(timeout=to))
    base_port = int(os.environ.get("LLMD_PD_BASE_PORT", "18200"))
    max_len = a.isl + a.osl + 64
    kt = {"kv_connector": "KvxConnector", "kv_role": "kv_producer" if is_prefill else "kv_consumer",
          "kv_load_failure_policy": "recompute",
          "kv_connector_extra_config": {"transport": os.environ.get("LLMD_KVX_TRANSPORT", "auto"),
                                        # a GPU bench never silently degrades a pull to TCP
                                        "require_ipc": a.device == "cuda"
                                        and os.environ.get("LLMD_KVX_TRANSPORT", "auto") == "auto"}}
    conc = a.concurrency * (1 if is_prefill else dtp)  # --concurrency is per GPU
    cfg = EngineConfig.create(
        a.model, device=a.device, block_size=a.block_size,
        max_num_seqs=max(conc, 8) if not is_prefill else 64,
        max_num_batched_tokens=a.max_num_batched_tokens, max_model_len=max_len,
        enforce_eager=a.enforce_eager or is_prefill or (dtp > 1 and os.environ.get("LLMD_BENCH_DEVICE") is not None),
        seed=a.seed, enable_prefix_caching=True,
        cuda_graph_max_bs=conc, kv_transfer_config=kt, gpu_memory_utilization=a.gpu_memory_utilization,
        kv_cache_memory_bytes=int(a.kv_cache_gb * 2**30) if a.kv_cache_gb else None,
        quantization=a.quantization, kv_cache_dtype=a.kv_cache_dtype)
    t0 = time.time()
    if is_follower:
        from llmd_amd.engine.tp_worker import run_follower

        n = run_follower(cfg, on_ready=lambda: dist.barrier(group=world_ctl))  # barrier: servers up
        log(rank, f"decode TP follower done after {n} steps")
        return None
    eng = LLMEngine(cfg, capture_graphs=not is_prefill)
    _sync(a)
    log(rank, f"{'prefill' if is_prefill else 'decode'} engine up in {time.time() - t0:.1f}s "
              f"({eng.runner.num_blocks} KV blocks)")
    if getattr(a, "pd_route", "router") == "router":
        return _run_routed(a, rank, world, P, dtp, drivers, is_prefill, eng, cfg, world_ctl, ctl, base_port, log)
    if is_prefill:
        srv_thread = _start_server(cfg, eng, base_port + rank)
        dist.barrier(group=world_ctl)        # servers up
        dist.barrier(group=ctl)              # decoders finished setup+warmup
        _sync(a)
        dist.barrier(group=ctl)              # timed region start
        dist.barrier(group=ctl)              # timed region end
        _sync(a)
        stats = [0.0, 0.0, 0.0]
        gathered = [None] * dist.get_world_size(ctl)
        dist.all_gather_object(gathered, {"elapsed": 0.0, "gen": 0, "ttft": [], "prefill": True,
                                          "prompt_tok": eng.metrics.n_prompt}, group=ctl)
        dist.barrier(group=ctl)
        srv_thread.stop()
        return _summarize(gathered, P, world, dtp)
    # ------------------------------------------------------------------ decode rank
    dist.barrier(group=world_ctl)  # prefill servers up
    prefill_urls = [f"http://127.0.0.1:{base_port + r}/v1/completions" for r in range(P)]
    sc = _SidecarThread(prefill_urls, a.model)
    vocab = cfg.model_config.vocab_size
    rng = np.random.default_rng(1234 + rank)
    issued = {}
    nreq = [0]

    def new_request(max_tokens):
        toks = rng.integers(100, vocab - 100, size=a.isl).tolist()
        nreq[0] += 1
        rid = f"d{rank}-{nreq[0]}"
        issued[rid] = (toks, max_tokens, time.monotonic())
        sc.submit(rid, toks)

    def drain_arrivals():
        n = 0
        while True:
            try:
                rid, ktp, ok = sc.results.get_nowait()
            except queue.Empty:
                return n
            toks, mt, t_issue = issued.pop(rid)
            eng.add_request(rid, toks, SamplingParams(max_tokens=mt, temperature=0.0, ignore_eos=True),
                            kv_transfer_params=ktp if ok else None, arrival_time=t_issue)
            n += 1

    in_flight = lambda: eng.sched.num_running + eng.sched.num_waiting + len(issued)  # noqa: E731

    def run_steps(n, until_full=False):
        k = 0
        while k < n:
            drain_arrivals()
            outs = eng.step()
            for o in outs:
                if o.finished:
                    new_request(a.osl)
            if eng.last_step_empty:
                time.sleep(0.0005)
                if not until_full:
                    continue  # an empty step is not a decode step
            k += 1

    for i in range(conc):
        new_request(max(1, int(a.osl * (i + 1) / conc)))
    ts = t_log = time.time()
    # setup: wait until the batch is filled and decoding
    while True:
        drain_arrivals()
        eng.step()
        if eng.last_step_empty:
            time.sleep(0.001)
        if not issued and eng.sched.num_waiting == 0 and all(r.output_token_ids for r in eng.sched.running):
            break
        if time.time() - ts > 1800:
            break
        if time.time() - t_log > 15:
            t_log = time.time()
            print(f"[bench-pd rank {rank}] setup {t_log - ts:.0f}s: issued={len(issued)} "
                  f"waiting={eng.sched.num_waiting} running={eng.sched.num_running} "
                  f"remote_wait={len(eng.sched.remote_wait)} gen={eng.metrics.n_gen}", flush=True)
    while in_flight() < conc:
        new_request(a.osl)
    log(rank, f"pd setup done in {time.time() - ts:.1f}s")
    run_steps(a.warmup)
    dist.barrier(group=ctl)
    eng.metrics.ttfts.clear()
    gen0 = eng.metrics.n_gen
    _sync(a)
    dist.barrier(group=ctl)
    t1 = time.perf_counter()
    run_steps(a.steps)
    _sync(a)
    dist.barrier(group=ctl)
    elapsed = time.perf_counter() - t1
    gen = eng.metrics.n_gen - gen0
    gathered = [None] * dist.get_world_size(ctl)
    kvm = getattr(eng.connector, "metrics", None) if getattr(eng, "connector", None) is not None else None
    dist.all_gather_object(gathered, {"elapsed": elapsed, "gen": gen, "ttft": list(eng.metrics.ttfts),
                                      "prefill": False, "kv_failures": int(getattr(kvm, "n_failed", 0))},
                           group=ctl)
    dist.barrier(group=ctl)
    sc.stop()
    eng.shutdown()  # releases the TP followers and the kvx agent
    return _summarize(gathered, P, world, dtp)


def _summarize(gathered, P, world, dtp=1):
    dec = [g for g in gathered if not g["prefill"]]
    el = max(g["elapsed"] for g in dec)
    tot = sum(g["gen"] for g in dec)
    tt = [t for g in gathered for t in g["ttft"]]
    out = {"elapsed": el, "gen": tot, "p50_ttft": statistics.median(tt) if tt else None,
           "prefill_ranks": P, "decode_ranks": world - P, "decode_tp": dtp, "n_ttft": len(tt),
           "kv_failures": sum(g.get("kv_failures", 0) for g in dec)}
    for g in gathered:  # routed path: rank 0 carries the client / router view
        for k in ("route", "open_loop", "router_pd_decisions", "ttft_p90", "steady_state", "ttft_source"):
            if k in g:
                out[k] = g[k]
    if any("sidecar_pd" in g for g in dec):
        out["sidecar_pd_requests"] = sum(g.get("sidecar_pd", 0) for g in dec)
        out["sidecar_fallbacks"] = sum(g.get("sidecar_fallbacks", 0) for g in dec)
    return out


class _SidecarThread:
    """Async HTTP client loop (routing-sidecar logic) on a private thread."""

    def __init__(self, urls, model):
        self.urls = urls
        self.model = model
        self.outstanding = [0] * len(urls)
        self.results: "queue.Queue[tuple]" = queue.Queue()
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self.loop.run_forever, daemon=True)
        self.thread.start()
        self.session = None

    def submit(self, rid, toks):
        asyncio.run_coroutine_threadsafe(self._one(rid, toks), self.loop)

    async def _one(self, rid, toks):
        import aiohttp

        if self.session is None:
            self.session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=3600))
        i = min(range(len(self.urls)), key=lambda k: self.outstanding[k])
        self.outstanding[i] += 1
        body = {"model": self.model, "prompt": toks, "max_tokens": 1, "temperature": 0.0, "stream": False,
                "kv_transfer_params": {"do_remote_decode": True, "do_remote_prefill": False}}
        try:
            async with self.session.post(self.urls[i], json=body, headers={"x-request-id": rid}) as r:
                d = await r.json()
                ktp = d.get("kv_transfer_params")
                self.results.put((rid, ktp, r.status == 200 and bool(ktp)))
        except Exception:  # noqa: BLE001 - prefill failure: decode-only fallback
            self.results.put((rid, None, False))
        finally:
            self.outstanding[i] -= 1

    def stop(self):
        async def close():
            if self.session:
                await self.session.close()
        asyncio.run_coroutine_threadsafe(close(), self.loop).result(timeout=10)
        self.loop.call_soon_threadsafe(self.loop.stop)


class _ServerThread(threading.Thread):
    def __init__(self, app, port):
        super().__init__(daemon=True)
        self.app, self.port = app, port
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        self.runner = None

    def run(self):
        from aiohttp import web

        asyncio.set_event_loop(self.loop)

        async def start():
            self.runner = web.AppRunner(self.app, access_log=None)
            await self.runner.setup()
            await web.TCPSite(self.runner, "127.0.0.1", self.port).start()
            self.ready.set()

        self.loop.run_until_complete(start())
        self.loop.run_forever()

    def stop(self):
        async def cleanup():
            await self.runner.cleanup()
        try:
            asyncio.run_coroutine_threadsafe(cleanup(), self.loop).result(timeout=10)
        except Exception:  # noqa: BLE001
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)


def _start_server(cfg, eng, port):
    from llmd_amd.serving.api_server import build_server

    srv = build_server(cfg, eng)
    t = _ServerThread(srv.app(), port)
    t.srv = srv
    t.start()
    t.ready.wait(60)
    orig_stop = t.stop

    def stop():
        orig_stop()
        srv.aeng.shutdown()
    t.stop = stop
    return t


# ============================================================================ routed P/D path
# The request path the reference benchmarks (guides/pd-disaggregation/README.md:331-470,
# router/pd-disaggregation.values.yaml:14-42): client -> router (EPP with the P/D
# EndpointPickerConfig: disagg-profile-handler + decider, prefill/decode filters and scorers)
# -> the chosen decode endpoint's routing sidecar (sidecar/routing_sidecar.py, nixlv2) ->
# prefill on the prefiller named in x-prefiller-host-port (max_tokens 1, do_remote_decode) ->
# decode on the local engine, which pulls the KV over kvx.
#   prefill rank r : OpenAI server on base + r (kv_producer)
#   decode driver d: OpenAI server on base + d (kv_consumer), routing sidecar on base + 500 + d
#   rank 0         : + the router (child process, python -m llmd_amd.router.proxy) on
#                    base + 1000 and the load client (closed loop for the timed window, then an
#                    open-loop Poisson phase for TTFT under queueing)
# Timing is unchanged: K decode steps on every decode driver between gloo barriers.


def _pd_router_config(decider: str) -> str:
    """The reference's P/D EndpointPickerConfig (deploy/router/pd-disaggregation-epp.yaml = the
    reference's router/pd-disaggregation.values.yaml:14-42), optionally with the load-aware decider."""
    import yaml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "deploy", "router", "pd-disaggregation-epp.yaml")) as f:
        cfg = yaml.safe_load(f)
    if decider == "load-aware":
        for pl in cfg["plugins"]:
            if pl.get("type") == "always-disagg-pd-decider":
                pl["type"] = "load-aware-pd-decider"
                pl["name"] = "always-disagg-pd-decider"  # keep the handler's reference
                pl["parameters"] = {"maxQueuedPromptTokens": int(os.environ.get("LLMD_PD_MAX_QUEUED", "65536"))}
    return yaml.safe_dump(cfg)


class _LoadClient:
    """Streaming OpenAI client on its own event loop thread (rank 0): a closed loop that keeps
    ``total`` requests in flight (a finished one is replaced at once), then an open-loop
    Poisson phase. TTFT = first streamed token - send time (the client's view: router, remote
    prefill, KV pull and the first decode step)."""

    def __init__(self, url, model, isl, vocab, seed=1234):
        self.url, self.model, self.isl, self.vocab = url, model, isl, vocab
        self.rng = np.random.default_rng(seed)
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self.loop.run_forever, daemon=True)
        self.thread.start()
        self.session = None
        self.closed = False
        self.osl = 1
        self.in_flight = 0
        self.first = 0          # requests of the closed loop that got their first token
        self.issued = 0
        self.events = []        # (t_send, t_first, n_tokens, t_end, ok)
        self.errors = 0

    def _call(self, coro):
        return asyncio.run_coroutine_threadsafe(coro, self.loop)

    async def _sess(self):
        import aiohttp

        if self.session is None:
            self.session = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0),
                                                 timeout=aiohttp.ClientTimeout(total=3600))
        return self.session

    async def _one(self, max_tokens, closed):
        s = await self._sess()
        toks = self.rng.integers(100, self.vocab - 100, size=self.isl).tolist()
        body = {"model": self.model, "prompt": toks, "max_tokens": int(max_tokens), "temperature": 0.0,
                "ignore_eos": True, "stream": True, "stream_options": {"include_usage": True}}
        self.in_flight += 1
        t0 = time.monotonic()
        t_first, n, ok = None, 0, False
        try:
            async with s.post(self.url, json=body) as r:
                if r.status == 200:
                    async for line in r.content:
                        if not line.startswith(b"data: ") or line.startswith(b"data: [DONE]"):
                            continue
                        d = json.loads(line[6:])
                        if d.get("choices") and t_first is None:
                            t_first = time.monotonic()
                            if closed:
                                self.first += 1
                        if d.get("usage"):
                            n = int(d["usage"].get("completion_tokens", 0))
                    ok = True
                else:
                    await r.read()
        except Exception:  # noqa: BLE001 - counted, never fatal to the bench
            pass
        self.in_flight -= 1
        if not ok:
            self.errors += 1
        self.events.append((t0, t_first, n, time.monotonic(), ok))
        if closed and self.closed:
            self.issued += 1
            self.loop.create_task(self._one(self.osl, True))

    def start_closed(self, total, osl):
        self.closed, self.osl = True, osl

        def go():
            for i in range(total):  # staggered lengths: completions spread over the first OSL steps
                self.issued += 1
                self.loop.create_task(self._one(max(1, int(osl * (i + 1) / total)), True))
        self.loop.call_soon_threadsafe(go)

    def stop_closed(self):
        self.closed = False

    def open_loop(self, rate, n):
        """Poisson arrivals at ``rate`` req/s, ``n`` requests; returns when all finished."""
        async def run():
            t_start = time.monotonic()
            k0 = len(self.events)
            tasks = []
            t = t_start
            for _ in range(n):
                t += float(self.rng.exponential(1.0 / rate))
                await asyncio.sleep(max(0.0, t - time.monotonic()))
                tasks.append(self.loop.create_task(self._one(self.osl, False)))
            await asyncio.gather(*tasks)
            return self.events[k0:], time.monotonic() - t_start
        return self._call(run()).result()

    def stop(self):
        async def close():
            if self.session:
                await self.session.close()
        try:
            self._call(close()).result(timeout=10)
        except Exception:  # noqa: BLE001
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)


def _sidecar_thread(decoder_url, port):
    from llmd_amd.sidecar.routing_sidecar import RoutingSidecar

    sc = RoutingSidecar(decoder_url)
    t = _ServerThread(sc.app(), port)
    t.sc = sc
    t.start()
    t.ready.wait(60)
    return t


def _scrape(url, timeout=5.0) -> str:
    import urllib.request

    with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310 - 127.0.0.1 only
        return r.read().decode()


def _counter_sum(text, name, label=None) -> float:
    """Sum of a prometheus counter's samples (``name_total{...}``; not ``_created``)."""
    tot = 0.0
    for line in text.splitlines():
        if (line.startswith(name + "_total{") or line.startswith(name + "{")) and (label is None or label in line):
            try:
                tot += float(line.rsplit(" ", 1)[1])
            except ValueError:
                pass
    return tot


def _run_routed(a, rank, world, P, dtp, drivers, is_prefill, eng, cfg, world_ctl, ctl, base, log):
    import subprocess

    from llmd_amd.tools import steady

    srv = _start_server(cfg, eng, base + rank)
    sc = _sidecar_thread(f"http://127.0.0.1:{base + rank}", base + 500 + rank) if not is_prefill else None
    dist.barrier(group=world_ctl)  # every server and sidecar up
    router = client = None
    n_dec_rep = len(drivers)
    total = a.concurrency * dtp * n_dec_rep  # --concurrency is per decode GPU
    if rank == 0:
        eps = [f"127.0.0.1:{base + r}:prefill" for r in range(P)] + \
              [f"127.0.0.1:{base + 500 + d}:decode" for d in drivers]
        rport = base + 1000
        env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        router = subprocess.Popen(
            [sys.executable, "-m", "llmd_amd.router.proxy", "--config-text",
             _pd_router_config(getattr(a, "pd_decider", "always")), "--endpoints", ",".join(eps),
             "--port", str(rport), "--metrics-port", str(rport + 1), "--failure-mode", "FailClose"],
            env=env, cwd=root, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        t0 = time.time()
        while True:
            try:
                _scrape(f"http://127.0.0.1:{rport}/health", timeout=1.0)
                break
            except Exception:  # noqa: BLE001 - not up yet
                if router.poll() is not None or time.time() - t0 > 120:
                    raise RuntimeError(f"router did not start: {router.stderr.read()[-2000:]!r}")
                time.sleep(0.2)
        log(rank, f"router up on {rport}: {len(eps)} endpoints ({P} prefill, {n_dec_rep} decode)")
        client = _LoadClient(f"http://127.0.0.1:{rport}/v1/completions", cfg.served_name, a.isl,
                             cfg.model_config.vocab_size)
        client.start_closed(total, a.osl)
        ts = time.time()
        while client.first < total and time.time() - ts < 1800:  # every slot decoding
            time.sleep(0.05)
        log(rank, f"routed setup: {total} requests decoding after {time.time() - ts:.1f}s "
                  f"(errors {client.errors})")
    dist.barrier(group=ctl)  # batch filled everywhere
    if not is_prefill:
        # steady state: completions re-spaced to R/OSL per step on this replica (tools/steady.py)
        fut = asyncio.run_coroutine_threadsafe(
            srv.srv.aeng.call(lambda e: steady.restagger(e.sched.running, a.osl, max(1, e.sched.num_running))),
            srv.loop)
        fut.result(timeout=120)

    def wait_steps(n):
        s0 = eng.step_count
        while eng.step_count < s0 + n:
            time.sleep(0.0005)

    if not is_prefill:
        wait_steps(a.warmup)
    dist.barrier(group=ctl)
    res = {"elapsed": 0.0, "gen": 0, "ttft": [], "prefill": is_prefill}
    _sync(a)
    dist.barrier(group=ctl)
    t1 = time.perf_counter()
    tm0 = time.monotonic()
    g0 = eng.metrics.n_gen
    if not is_prefill:
        wait_steps(a.steps)
        _sync(a)
    dist.barrier(group=ctl)
    tm1 = time.monotonic()
    if not is_prefill:
        res["elapsed"] = time.perf_counter() - t1
        res["gen"] = eng.metrics.n_gen - g0
        kvm = getattr(eng.connector, "metrics", None) if getattr(eng, "connector", None) is not None else None
        res["kv_failures"] = int(getattr(kvm, "n_failed", 0))
        res["sidecar_pd"] = int(sc.sc.m_req.labels("pd")._value.get())
        res["sidecar_fallbacks"] = int(sum(c._value.get() for c in sc.sc.m_fallback._metrics.values()))
    if rank == 0:
        win = [(e[1] - e[0]) for e in client.events if e[1] is not None and tm0 <= e[1] <= tm1]
        res["ttft"] = win
        if win:
            res["ttft_p90"] = float(np.percentile(win, 90))
        res["route"] = "client -> router (EPP, reference P/D config) -> decode sidecar -> prefill + kvx pull"
        done = sum(1 for e in client.events if tm0 <= e[3] <= tm1 and e[4])
        res["steady_state"] = {"completions_in_window": done,
                               "conservation_completions": round(a.steps * total / a.osl, 2)}
    gathered = [None] * dist.get_world_size(ctl)
    dist.all_gather_object(gathered, res, group=ctl)
    if rank == 0:
        out = _summarize(gathered, P, world, dtp)
        # open loop (the reference's rate-driven benchmark): Poisson arrivals at a rate below the
        # closed loop's completion rate, after the closed loop drained; TTFT under queueing
        client.stop_closed()
        td = time.time()
        while client.in_flight > 0 and time.time() - td < 600:
            time.sleep(0.05)
        closed_rate = out["gen"] / out["elapsed"] / a.osl if out["elapsed"] > 0 else 0.0
        rate = float(getattr(a, "open_loop_rate", 0.0) or 0.0) or 0.9 * closed_rate
        n_req = int(getattr(a, "open_loop_requests", 0) or 0) or max(8, min(400, int(rate * 20)))
        if rate > 0:
            evs, dur = client.open_loop(rate, n_req)
            tt = [e[1] - e[0] for e in evs if e[1] is not None]
            toks = sum(e[2] for e in evs)
            out["open_loop"] = {"rate_req_s": round(rate, 3), "requests": n_req, "duration_s": round(dur, 2),
                                "ttft_p50_s": round(statistics.median(tt), 4) if tt else None,
                                "ttft_p90_s": round(float(np.percentile(tt, 90)), 4) if tt else None,
                                "output_tok_s": round(toks / dur, 1) if dur > 0 else None,
                                "errors": sum(1 for e in evs if not e[4])}
        # p50 TTFT: the closed-loop window's when it saw enough first tokens, else the open loop's
        # (the reference's TTFT comes from its rate-driven run)
        out["ttft_source"] = "closed-loop window"
        if out.get("n_ttft", 0) < 5 and out.get("open_loop", {}).get("ttft_p50_s") is not None:
            out["p50_ttft"] = out["open_loop"]["ttft_p50_s"]
            out["ttft_p90"] = out["open_loop"]["ttft_p90_s"]
            out["ttft_source"] = "open-loop phase"
        try:
            m = _scrape(f"http://127.0.0.1:{base + 1001}/metrics")
            out["router_pd_decisions"] = {k: _counter_sum(m, "llm_d_router_epp_pd_decision", f'decision_type="{k}"')
                                          for k in ("disagg", "decode-only")}
        except Exception as e:  # noqa: BLE001
            out["router_pd_decisions"] = {"error": repr(e)[:200]}
        log(rank, f"routed P/D: {out.get('router_pd_decisions')}, open loop {out.get('open_loop')}")
    else:
        out = None
    dist.barrier(group=ctl)  # rank 0's open-loop phase done
    if client is not None:
        client.stop()
    if router is not None:
        router.terminate()
        try:
            router.wait(10)
        except subprocess.TimeoutExpired:
            router.kill()
    if sc is not None:
        sc.stop()
    srv.stop()
    if not is_prefill:
        eng.shutdown()
    return out
