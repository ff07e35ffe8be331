"""Benchmark harness / load generator (reference helpers/benchmark.md,
workload config shape of guides/wide-ep-lws/experimental-dp-aware/benchmarks/
bench-multi-turn/config.yaml - the inference-perf schema).

Config (YAML or dict)::

  load:   {type: constant|poisson|concurrent, stages: [{rate, duration} | {concurrency, num_requests}]}
  api:    {type: completion|chat, streaming: true}
  server: {base_url, model_name, ignore_eos}
  data:   {type: random, input_distribution: {mean, std, min, max},
                         output_distribution: {mean, std, min, max}}
        | {type: shared_prefix, shared_prefix: {num_groups, num_prompts_per_group,
                         system_prompt_len, question_len, output_len, enable_multi_turn_chat}}

Prompts are token-ID arrays (no tokenizer needed; exact lengths). Every
request is streamed; per request we record TTFT, inter-token gaps, e2e,
output tokens. The report follows the cross-harness ``benchmark_report``
layout: per-stage and summary ``{requests, latency{time_to_first_token,
inter_token_latency, time_per_output_token, request_latency}{mean,p50,p90,
p95,p99,units}, throughput{requests_per_sec, input_tokens_per_sec,
output_tokens_per_sec, total_tokens_per_sec}}``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import sys
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np


@dataclass
class Req:
    prompt: list
    max_tokens: int
    group: int = -1
    history_key: Optional[tuple] = None


@dataclass
class Result:
    ok: bool
    ttft: float = 0.0
    e2e: float = 0.0
    itls: list = field(default_factory=list)
    n_in: int = 0
    n_out: int = 0
    err: str = ""
    t_start: float = 0.0


# ------------------------------------------------------------------- data
class RandomData:
    def __init__(self, cfg: dict, vocab: int = 32000, seed: int = 0):
        self.i = cfg.get("input_distribution", {"mean": 512})
        self.o = cfg.get("output_distribution", {"mean": 128})
        self.vocab = vocab
        self.rng = np.random.default_rng(seed)

    def _len(self, d) -> int:
        x = self.rng.normal(d["mean"], d.get("std", 0.0)) if d.get("std") else d["mean"]
        return int(np.clip(round(x), d.get("min", 1), d.get("max", 1 << 20)))

    def next(self) -> Req:
        return Req(self.rng.integers(100, self.vocab - 100, size=self._len(self.i)).tolist(), self._len(self.o))


class SharedPrefixData:
    """num_groups system prompts x num_prompts_per_group unique questions;
    optional multi-turn: each user's context grows with its previous turns."""

    def __init__(self, cfg: dict, vocab: int = 32000, seed: int = 0):
        c = cfg["shared_prefix"]
        self.rng = np.random.default_rng(seed)
        self.vocab = vocab
        self.G, self.P = int(c.get("num_groups", 10)), int(c.get("num_prompts_per_group", 10))
        self.out = int(c.get("output_len", 128))
        self.multi = bool(c.get("enable_multi_turn_chat", False))
        tok = lambda n: self.rng.integers(100, vocab - 100, size=int(n)).tolist()  # noqa: E731
        self.prefix = [tok(c.get("system_prompt_len", 1024)) for _ in range(self.G)]
        self.questions = [[tok(c.get("question_len", 128)) for _ in range(self.P)] for _ in range(self.G)]
        self.history: dict[tuple, list] = {}
        self.k = 0

    def next(self) -> Req:
        g, p = self.k % self.G, (self.k // self.G) % self.P
        self.k += 1
        key = (g, p)
        ctx = self.history.get(key, []) if self.multi else []
        prompt = self.prefix[g] + ctx + self.questions[g][p]
        return Req(prompt, self.out, g, key if self.multi else None)

    def record_turn(self, req: Req, out_tokens: int):
        if req.history_key is not None:
            h = self.history.setdefault(req.history_key, [])
            h += self.questions[req.history_key[0]][req.history_key[1]] + \
                self.rng.integers(100, self.vocab - 100, size=out_tokens).tolist()


def make_data(cfg: dict, vocab: int, seed: int):
    t = cfg.get("type", "random")
    return SharedPrefixData(cfg, vocab, seed) if t == "shared_prefix" else RandomData(cfg, vocab, seed)


# ----------------------------------------------------------------- client
async def send(session, base_url: str, model: str, api: str, req: Req, ignore_eos: bool) -> Result:
    t0 = time.perf_counter()
    res = Result(ok=False, n_in=len(req.prompt), t_start=time.time())
    if api == "chat":
        # token-id prompts are not expressible in chat; send a placeholder text of similar size
        url = base_url + "/v1/chat/completions"
        body = {"model": model, "messages": [{"role": "user", "content": " ".join(map(str, req.prompt))}],
                "max_tokens": req.max_tokens, "stream": True, "stream_options": {"include_usage": True}}
    else:
        url = base_url + "/v1/completions"
        body = {"model": model, "prompt": req.prompt, "max_tokens": req.max_tokens, "stream": True,
                "stream_options": {"include_usage": True}}
    if ignore_eos:
        body["ignore_eos"] = True
    last = None
    n_chunks = 0
    try:
        async with session.post(url, json=body) as r:
            if r.status != 200:
                res.err = f"http {r.status}: {(await r.text())[:200]}"
                return res
            async for raw in r.content:
                line = raw.strip()
                if not line.startswith(b"data:"):
                    continue
                data = line[5:].strip()
                if data == b"[DONE]":
                    break
                d = json.loads(data)
                if d.get("usage"):
                    res.n_out = d["usage"].get("completion_tokens", res.n_out)
                if not d.get("choices"):
                    continue
                now = time.perf_counter()
                if last is None:
                    res.ttft = now - t0
                else:
                    res.itls.append(now - last)
                last = now
                n_chunks += 1
        res.e2e = time.perf_counter() - t0
        res.n_out = res.n_out or n_chunks
        res.ok = last is not None
    except Exception as e:  # noqa: BLE001
        res.err = str(e)
    return res


def _stats(xs: list[float], units: str = "s") -> dict:
    if not xs:
        return {"mean": None, "p50": None, "p90": None, "p95": None, "p99": None, "units": units}
    a = np.asarray(xs)
    return {"mean": float(a.mean()), "p50": float(np.percentile(a, 50)), "p90": float(np.percentile(a, 90)),
            "p95": float(np.percentile(a, 95)), "p99": float(np.percentile(a, 99)), "min": float(a.min()),
            "max": float(a.max()), "units": units}


def summarize(results: list[Result], duration: float) -> dict:
    ok = [r for r in results if r.ok]
    tpot = [(r.e2e - r.ttft) / (r.n_out - 1) for r in ok if r.n_out > 1]
    n_in, n_out = sum(r.n_in for r in ok), sum(r.n_out for r in ok)
    return {
        "requests": {"total": len(results), "failures": len(results) - len(ok),
                     "input_length": _stats([r.n_in for r in ok], "tokens"),
                     "output_length": _stats([r.n_out for r in ok], "tokens")},
        "latency": {"time_to_first_token": _stats([r.ttft for r in ok]),
                    "inter_token_latency": _stats([x for r in ok for x in r.itls]),
                    "time_per_output_token": _stats(tpot),
                    "request_latency": _stats([r.e2e for r in ok])},
        "throughput": {"requests_per_sec": len(ok) / duration if duration else 0.0,
                       "input_tokens_per_sec": n_in / duration if duration else 0.0,
                       "output_tokens_per_sec": n_out / duration if duration else 0.0,
                       "total_tokens_per_sec": (n_in + n_out) / duration if duration else 0.0},
        "duration_s": duration,
    }


# ------------------------------------------------------------------ runner
def per_request(results: list[Result], stage: int) -> list[dict]:
    """inference-perf style per-request lifecycle records."""
    return [{"stage": stage, "start_time": r.t_start, "end_time": r.t_start + r.e2e, "ok": r.ok,
             "error": r.err or None, "prompt_tokens": r.n_in, "output_tokens": r.n_out,
             "time_to_first_token": r.ttft if r.ok else None, "inter_token_latencies": r.itls,
             "request_latency": r.e2e if r.ok else None} for r in results]


async def run(cfg: dict, vocab: int = 32000, seed: int = 0, records: bool = False) -> dict:
    import aiohttp

    load, server, api = cfg.get("load", {}), cfg["server"], cfg.get("api", {}).get("type", "completion")
    base = server["base_url"].rstrip("/")
    model = server.get("model_name", "model")
    ignore_eos = bool(server.get("ignore_eos", True))
    data = make_data(cfg.get("data", {}), vocab, seed)
    rng = random.Random(seed)
    stages_out = []
    recs: list[dict] = []
    all_res: list[Result] = []
    t_all = time.perf_counter()
    conn = aiohttp.TCPConnector(limit=0)
    async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=None)) as s:
        async def one(q: Req, sink: list):
            r = await send(s, base, model, api, q, ignore_eos)
            if isinstance(data, SharedPrefixData):
                data.record_turn(q, r.n_out)
            sink.append(r)

        for i, st in enumerate(load.get("stages", [{"rate": 1, "duration": 10}])):
            res: list[Result] = []
            t0 = time.perf_counter()
            typ = load.get("type", "constant")
            if typ == "concurrent":
                n_total = int(st.get("num_requests", 100))
                conc = int(st.get("concurrency", 8))
                counter = {"n": 0}

                async def worker():
                    while counter["n"] < n_total:
                        counter["n"] += 1
                        await one(data.next(), res)
                await asyncio.gather(*[worker() for _ in range(conc)])
            else:
                rate, dur = float(st["rate"]), float(st["duration"])
                tasks = []
                t_next = 0.0
                while t_next < dur:
                    delay = t0 + t_next - time.perf_counter()
                    if delay > 0:
                        await asyncio.sleep(delay)
                    tasks.append(asyncio.ensure_future(one(data.next(), res)))
                    t_next += rng.expovariate(rate) if typ == "poisson" else 1.0 / rate
                await asyncio.gather(*tasks)
            dt = time.perf_counter() - t0
            stages_out.append({"stage": i, "config": st, **summarize(res, dt)})
            if records:
                recs += per_request(res, i)
            all_res += res
    out = {"version": "0.1", "harness": "llmd-loadgen", "scenario": cfg, "stages": stages_out,
           "summary": summarize(all_res, time.perf_counter() - t_all)}
    if records:
        out["per_request"] = recs
    return out


def main(argv=None):
    import yaml

    p = argparse.ArgumentParser("llmd-loadgen")
    p.add_argument("--config", required=True, help="inference-perf style YAML")
    p.add_argument("--base-url")
    p.add_argument("--model")
    p.add_argument("--vocab", type=int, default=32000)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--output", default="-")
    a = p.parse_args(argv)
    with open(a.config) as f:
        cfg = yaml.safe_load(f)
    if a.base_url:
        cfg.setdefault("server", {})["base_url"] = a.base_url
    if a.model:
        cfg.setdefault("server", {})["model_name"] = a.model
    rep = asyncio.run(run(cfg, a.vocab, a.seed))
    txt = yaml.safe_dump(rep, sort_keys=False)
    if a.output == "-":
        sys.stdout.write(txt)
    else:
        with open(a.output, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
