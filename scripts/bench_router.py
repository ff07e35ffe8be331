"""Router overhead: what the EPP + Python streaming proxy add per request, and
the proxy's streaming ceiling, at 8+ endpoints (no GPU: engines are the
simulator, llmd_amd/sim/server.py, with ~zero prefill time and a 1 ms decode
step so the proxy, not the engines, is the bottleneck).

A. EPP decision latency in process (parse -> flow control -> producers ->
   filters/scorers -> pick; DEFAULT_CONFIG: queue + kv-util + prefix + no-hit-lru
   scorers), N endpoints with live-looking metrics, 2 KB prompts sharing
   prefixes: p50/p99 microseconds per decision.
B. End to end: E simulator processes, the router (llmd_amd.router.proxy) in its
   own process, P client processes at total concurrency C issuing streaming
   completions (``max_tokens`` chunks each): requests/s, streamed chunks/s and
   TTFT p50/p99 through the router vs the same load sent straight to the engines
   (round robin) - the difference is the router's added latency.

  python scripts/bench_router.py [--endpoints 8] [--conc 64,256] [--secs 8] [--workers 1,py4,native4]
      [--out profiles/router_overhead.json]

``--workers``: data planes in front of one EPP process (router/workers.py):
``1`` the in-process Python proxy, ``pyN`` N aiohttp worker processes,
``nativeN`` the llmd-relay executable with N epoll threads
(csrc/relay/relay.cpp); each is measured against the same direct baseline.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


# ---------------------------------------------------------------- A: EPP decision latency
def bench_epp(n_endpoints: int, n_req: int = 3000) -> dict:
    import random

    from llmd_amd.router.api import ControlPlane
    from llmd_amd.router.datalayer import EndpointStore, endpoints_from_yaml
    from llmd_amd.router.epp import EPP
    from llmd_amd.router.proxy import DEFAULT_CONFIG

    async def run():
        store = EndpointStore()
        epp = EPP(DEFAULT_CONFIG, store, ControlPlane(), "pool")
        eps = [{"name": f"ep{i}", "address": "10.0.0.%d" % (i + 1), "port": 8000} for i in range(n_endpoints)]
        for e in endpoints_from_yaml({"endpoints": eps}):
            await store.add(e)
        rnd = random.Random(0)
        from llmd_amd.router.plugins.scheduling import KV_USAGE, RUNNING, WAITING

        for e in store.all():  # live-looking scraped metrics
            e.attrs.update({WAITING: rnd.randint(0, 8), RUNNING: rnd.randint(0, 64), KV_USAGE: rnd.random()})
        prefixes = ["".join(rnd.choice("abcdefghij ") for _ in range(1500)) for _ in range(32)]
        lat = []
        for i in range(n_req):
            body = json.dumps({"model": "m", "prompt": prefixes[i % 32] + str(i) * 50, "max_tokens": 16,
                               "stream": True}).encode()
            t0 = time.perf_counter()
            d = await epp.handle("/v1/completions", body, {"content-type": "application/json"})
            lat.append((time.perf_counter() - t0) * 1e6)
            epp.on_response_headers(d, 200, {})
            epp.on_response_complete(d, {"status": 200, "ttft": 0.01, "duration": 0.02,
                                         "usage": {"prompt_tokens": 400, "completion_tokens": 16}})
        await epp.stop()
        return lat

    lat = asyncio.run(run())[200:]  # drop warm-up
    return {"endpoints": n_endpoints, "decisions": len(lat), "p50_us": round(_pct(lat, 0.5), 1),
            "p99_us": round(_pct(lat, 0.99), 1), "mean_us": round(statistics.mean(lat), 1),
            "max_decisions_per_s": round(1e6 / statistics.mean(lat))}


# ---------------------------------------------------------------- B: end to end
def _client(targets, conc, secs, max_tokens, q):
    import aiohttp

    async def run():
        ttft, n_req, n_chunks, errors = [], 0, 0, 0
        stop = time.monotonic() + secs
        conn = aiohttp.TCPConnector(limit=0)
        async with aiohttp.ClientSession(connector=conn) as s:
            async def worker(w):
                nonlocal n_req, n_chunks, errors
                i = w
                while time.monotonic() < stop:
                    url = targets[i % len(targets)]
                    i += conc
                    # distinct prompts: no prefix affinity, so routing spreads the load like round robin
                    body = {"model": "sim-model", "prompt": f"{os.getpid()}-{w}-{i} " + "x" * 200,
                            "max_tokens": max_tokens, "stream": True}
                    t0 = time.monotonic()
                    first = None
                    try:
                        async with s.post(url, json=body) as r:
                            if r.status != 200:
                                errors += 1
                                await r.read()
                                continue
                            async for _ in r.content.iter_any():
                                if first is None:
                                    first = time.monotonic()
                                n_chunks += 1
                        n_req += 1
                        ttft.append((first or time.monotonic()) - t0)
                    except aiohttp.ClientError:
                        errors += 1
            await asyncio.gather(*[worker(w) for w in range(conc)])
        return ttft, n_req, n_chunks, errors

    q.put(asyncio.run(run()))


def _load(targets, conc, secs, max_tokens, procs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    per = max(1, conc // procs)
    ps = [ctx.Process(target=_client, args=(targets, per, secs, max_tokens, q)) for _ in range(procs)]
    t0 = time.monotonic()
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    wall = time.monotonic() - t0
    ttft = [x for r in res for x in r[0]]
    n_req = sum(r[1] for r in res)
    return {"conc": per * procs, "req_s": round(n_req / secs, 1), "chunks_s": round(sum(r[2] for r in res) / secs),
            "errors": sum(r[3] for r in res), "ttft_p50_ms": round(_pct(ttft, 0.5) * 1e3, 2),
            "ttft_p99_ms": round(_pct(ttft, 0.99) * 1e3, 2), "wall_s": round(wall, 1)}


def _wait_port(port, timeout=60):
    t = time.time() + timeout
    while time.time() < t:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return
        except OSError:
            time.sleep(0.2)
    raise RuntimeError(f"port {port} never opened")


def _plane(spec: str):
    """'1' -> in-process Python proxy; 'pyN' -> N Python worker processes; 'nativeN' -> the
    llmd-relay data plane with N threads (csrc/relay/relay.cpp)."""
    if spec.startswith("native"):
        return "native", int(spec[6:])
    if spec.startswith("py"):
        return "python", int(spec[2:])
    return ("python" if int(spec) > 1 else "inproc"), int(spec)


def _start_router(env, ports, spec):
    plane, workers = _plane(spec)
    rport, mport = _free_port(), _free_port()
    extra = ["--data-plane", plane] if plane != "inproc" else []
    router = subprocess.Popen([sys.executable, "-m", "llmd_amd.router.proxy", "--port", str(rport),
                               "--metrics-port", str(mport), "--workers", str(workers),
                               "--endpoints", ",".join(f"127.0.0.1:{p}" for p in ports), "--v", "0"] + extra,
                              env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return router, rport


def _stop(procs):
    for p in procs:
        p.terminate()
    for p in procs:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()


def bench_e2e(n_endpoints, concs, secs, max_tokens, procs, workers=("1",)) -> list:
    env = dict(os.environ, PYTHONPATH=ROOT)
    ports = [_free_port() for _ in range(n_endpoints)]
    sims = [subprocess.Popen([sys.executable, "-m", "llmd_amd.sim.server", "--port", str(p), "--max-num-seqs", "4096",
                              "--prefill-tps", "1e9", "--decode-step-ms", "1"], env=env,
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL) for p in ports]
    out = []
    try:
        for p in ports:
            _wait_port(p)
        direct = [f"http://127.0.0.1:{p}/v1/completions" for p in ports]
        base = {c: _load(direct, c, secs, max_tokens, procs) for c in concs}
        for w in workers:
            router, rport = _start_router(env, ports, w)
            try:
                _wait_port(rport)
                time.sleep(2.0)  # first metrics scrape, workers up
                routed = [f"http://127.0.0.1:{rport}/v1/completions"]
                for c in concs:
                    d = base[c]
                    r = _load(routed, c, secs, max_tokens, procs)
                    row = {"endpoints": n_endpoints, "router_workers": _plane(w)[1], "data_plane": _plane(w)[0],
                           "conc": c, "max_tokens": max_tokens,
                           "direct": d, "routed": r,
                           "added_ttft_p50_ms": round(r["ttft_p50_ms"] - d["ttft_p50_ms"], 2),
                           "added_ttft_p99_ms": round(r["ttft_p99_ms"] - d["ttft_p99_ms"], 2),
                           "routed_vs_direct_req_s": round(r["req_s"] / max(d["req_s"], 1e-9), 3)}
                    print(json.dumps(row), flush=True)
                    out.append(row)
            finally:
                _stop([router])
    finally:
        _stop(sims)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--endpoints", type=int, default=8)
    ap.add_argument("--conc", default="64,256")
    ap.add_argument("--secs", type=float, default=8.0)
    ap.add_argument("--max-tokens", type=int, default=32)
    ap.add_argument("--procs", type=int, default=3, help="client processes")
    ap.add_argument("--skip-e2e", action="store_true")
    ap.add_argument("--workers", default="1,py4,native4",
                    help="data planes to compare: 1 (in-process Python proxy), pyN (N Python worker "
                         "processes), nativeN (llmd-relay with N threads)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {"cpus": os.cpu_count(), "epp": [bench_epp(n) for n in (a.endpoints, 4 * a.endpoints)]}
    for r in res["epp"]:
        print(json.dumps({"epp_decision": r}), flush=True)
    if not a.skip_e2e:
        res["e2e"] = bench_e2e(a.endpoints, [int(c) for c in a.conc.split(",")], a.secs, a.max_tokens, a.procs,
                               a.workers.split(","))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
