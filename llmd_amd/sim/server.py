"""GPU-free engine simulator (the llm-d-inference-sim analogue; SURVEY §4
item 3, BASELINE config #1 "router plumbing, no GPU").

Speaks the same contract as the real engine: OpenAI completions/chat
(stream + non-stream), /health, /v1/models, vLLM-named /metrics, KV events
(real chained block hashes through the native BlockManager, so precise
prefix routing works end to end), /v1/completions/render, and the P/D
``kv_transfer_params`` protocol (prefill role returns remote params; decode
role "pulls" with a configurable transfer delay).

Latency model (per request):
  TTFT = queue wait + uncached_prompt_tokens / prefill_tps
  ITL  = decode_step_s * (1 + running / batch_knee)
A concurrency limit (--max-num-seqs) creates real queueing, so saturation
detectors and flow control see meaningful telemetry.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import random
import time
import uuid
from typing import Optional

import numpy as np
from aiohttp import web

from llmd_amd import _rt_loader
from llmd_amd.engine.metrics import EngineMetrics
from llmd_amd.serving.tokenizer import ByteTokenizer, render_chat

log = logging.getLogger("llmd.sim")


class SimEngine:
    def __init__(self, model="sim-model", block_size=16, num_blocks=4096, max_num_seqs=64,
                 prefill_tps=20000.0, decode_step_s=0.01, batch_knee=64, role="both",
                 kv_events_port: Optional[int] = None, topic: Optional[str] = None, transfer_s=0.002,
                 fail_prefill: float = 0.0, max_lora=0, vocab=32000):
        self.model = model
        self.bs = block_size
        self.bm = _rt_loader.rt().BlockManager(num_blocks, block_size, True, True)
        self.metrics = EngineMetrics(model, block_size, num_blocks, max_lora=max_lora)
        self.sem = asyncio.Semaphore(max_num_seqs)
        self.max_num_seqs = max_num_seqs
        self.prefill_tps, self.decode_step_s, self.knee = prefill_tps, decode_step_s, batch_knee
        self.role = role
        self.running = 0
        self.waiting = 0
        self.tok = ByteTokenizer(vocab)
        self.transfer_s = transfer_s
        self.fail_prefill = fail_prefill
        self.held: dict[str, tuple[int, float]] = {}
        self.pub = None
        if kv_events_port is not None:
            from llmd_amd.serving.kv_events import KVEventPublisher

            self.pub = KVEventPublisher(f"tcp://*:{kv_events_port}", topic or f"kv@127.0.0.1:0@{model}", block_size)
        self.loras: set[str] = set()
        self.max_lora = max_lora
        self.paused = False

    def _flush(self):
        ev = self.bm.take_events()
        if ev and self.pub is not None:
            self.pub.publish(ev)

    def _update_gauges(self):
        m = self.metrics
        m.running.labels(self.model).set(self.running)
        m.waiting.labels(self.model).set(self.waiting)
        m.kv_usage.labels(self.model).set(self.bm.usage())

    async def generate(self, prompt_ids: list[int], max_tokens: int, ktp: Optional[dict] = None):
        """Yields (token_id, is_last, extra) with simulated timing."""
        seq = random.getrandbits(62)
        t_arr = time.monotonic()
        self.waiting += 1
        self._update_gauges()
        async with self.sem:
            self.waiting -= 1
            self.running += 1
            self._update_gauges()
            try:
                toks = np.asarray(prompt_ids, dtype=np.int32)
                if ktp and ktp.get("do_remote_prefill"):
                    blocks = self.bm.allocate_remote(seq, len(prompt_ids), 0)
                    await asyncio.sleep(self.transfer_s + len(prompt_ids) * 2e-7)
                    cached = len(prompt_ids)
                    self.bm.commit(seq, toks, len(prompt_ids))
                else:
                    cached = self.bm.acquire(seq, toks, 0)
                    self.bm.grow(seq, len(prompt_ids) + max_tokens)
                    await asyncio.sleep(max(0, len(prompt_ids) - cached) / self.prefill_tps)
                    self.bm.commit(seq, toks, len(prompt_ids))
                self._flush()
                self.metrics.prompt_tokens.labels(self.model).inc(len(prompt_ids) - cached)
                self.metrics.ttft.labels(self.model).observe(time.monotonic() - t_arr)
                for i in range(max_tokens):
                    if i > 0:
                        await asyncio.sleep(self.decode_step_s * (1 + self.running / self.knee))
                    self.metrics.gen_tokens.labels(self.model).inc()
                    yield 3 + (hash((seq, i)) % 200), i == max_tokens - 1, {"cached": cached}
            finally:
                if ktp and ktp.get("do_remote_decode"):
                    self.held[str(seq)] = (seq, time.monotonic())
                else:
                    self.bm.free(seq)
                self.running -= 1
                self._update_gauges()
                self._flush()


def make_app(eng: SimEngine) -> web.Application:
    app = web.Application()

    async def health(req):
        return web.Response(text="")

    async def models(req):
        data = [{"id": eng.model, "object": "model", "owned_by": "llmd-sim"}]
        data += [{"id": n, "object": "model", "parent": eng.model} for n in sorted(eng.loras)]
        return web.json_response({"object": "list", "data": data})

    async def metrics(req):
        eng._update_gauges()
        if eng.max_lora:
            eng.metrics.set_lora(sorted(eng.loras), [])
        return web.Response(body=eng.metrics.render(), content_type="text/plain")

    def ids_of(body):
        if "messages" in body:
            return eng.tok.encode(render_chat(body["messages"]))
        p = body.get("prompt", "")
        if isinstance(p, list) and p and isinstance(p[0], int):
            return list(p)
        if isinstance(p, list):
            p = "".join(map(str, p))
        return eng.tok.encode(p)

    async def render(req):
        body = await req.json()
        ids = ids_of(body)
        return web.json_response({"token_ids": ids, "prompt_token_ids": ids, "count": len(ids)})

    async def serve(req: web.Request):
        body = await req.json()
        chat = req.path.endswith("chat/completions")
        ids = ids_of(body)
        mt = int(body.get("max_tokens") or body.get("max_completion_tokens") or 16)
        ktp = body.get("kv_transfer_params")
        rid = req.headers.get("x-request-id") or f"cmpl-{uuid.uuid4().hex}"
        if ktp and ktp.get("do_remote_decode") and random.random() < eng.fail_prefill:
            return web.json_response({"error": {"message": "injected prefill failure"}}, status=500)
        stream = bool(body.get("stream"))
        out_ktp = None
        if ktp and ktp.get("do_remote_decode"):
            out_ktp = {"do_remote_prefill": True, "do_remote_decode": False, "remote_engine_id": "sim",
                       "remote_host": req.host.split(":")[0], "remote_port": 0,
                       "remote_block_ids": [], "remote_request_id": rid}
        obj = "chat.completion.chunk" if chat else "text_completion"
        if stream:
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
            await resp.prepare(req)
            n = 0
            async for tok, last, extra in eng.generate(ids, mt, ktp):
                n += 1
                txt = chr(97 + tok % 26)
                ch = {"index": 0, "finish_reason": "length" if last else None}
                ch.update({"delta": {"content": txt}} if chat else {"text": txt})
                await resp.write(b"data: " + json.dumps({"id": rid, "object": obj, "model": eng.model,
                                                         "choices": [ch]}).encode() + b"\n\n")
            if (body.get("stream_options") or {}).get("include_usage"):
                await resp.write(b"data: " + json.dumps({"id": rid, "object": obj, "choices": [], "usage": {
                    "prompt_tokens": len(ids), "completion_tokens": n, "total_tokens": len(ids) + n,
                    "prompt_tokens_details": {"cached_tokens": extra.get("cached", 0)}}}).encode() + b"\n\n")
            await resp.write(b"data: [DONE]\n\n")
            await resp.write_eof()
            return resp
        text, n, cached = "", 0, 0
        async for tok, last, extra in eng.generate(ids, mt, ktp):
            text += chr(97 + tok % 26)
            n += 1
            cached = extra.get("cached", 0)
        ch = {"index": 0, "finish_reason": "length"}
        ch.update({"message": {"role": "assistant", "content": text}} if chat else {"text": text})
        out = {"id": rid, "object": "chat.completion" if chat else "text_completion", "model": eng.model,
               "choices": [ch], "usage": {"prompt_tokens": len(ids), "completion_tokens": n,
                                          "total_tokens": len(ids) + n,
                                          "prompt_tokens_details": {"cached_tokens": cached}}}
        if out_ktp is not None:
            out["kv_transfer_params"] = out_ktp
        return web.json_response(out)

    async def load_lora(req):
        body = await req.json()
        if eng.max_lora and len(eng.loras) >= eng.max_lora:
            return web.json_response({"error": "max loras"}, status=400)
        eng.loras.add(body["lora_name"])
        return web.Response(text="ok")

    app.router.add_get("/health", health)
    app.router.add_get("/v1/models", models)
    app.router.add_get("/metrics", metrics)
    app.router.add_post("/v1/completions", serve)
    app.router.add_post("/v1/chat/completions", serve)
    app.router.add_post("/v1/completions/render", render)
    app.router.add_post("/v1/chat/completions/render", render)
    app.router.add_post("/v1/load_lora_adapter", load_lora)
    return app


async def start_sim(port: int = 0, host: str = "127.0.0.1", **kw):
    """Start a simulator in the running loop; returns (runner, engine, port)."""
    eng = SimEngine(**kw)
    runner = web.AppRunner(make_app(eng), access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    real_port = site._server.sockets[0].getsockname()[1]
    return runner, eng, real_port


def main(argv=None):
    p = argparse.ArgumentParser("llmd-amd engine simulator")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--model", default="sim-model")
    p.add_argument("--block-size", type=int, default=16)
    p.add_argument("--num-blocks", type=int, default=4096)
    p.add_argument("--max-num-seqs", type=int, default=64)
    p.add_argument("--prefill-tps", type=float, default=20000.0)
    p.add_argument("--decode-step-ms", type=float, default=10.0)
    p.add_argument("--role", default="both", choices=["both", "prefill", "decode"])
    p.add_argument("--kv-events-port", type=int, default=None)
    p.add_argument("--max-lora", type=int, default=0)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)

    async def run():
        await start_sim(a.port, "0.0.0.0", model=a.model, block_size=a.block_size, num_blocks=a.num_blocks,
                        max_num_seqs=a.max_num_seqs, prefill_tps=a.prefill_tps,
                        decode_step_s=a.decode_step_ms / 1000, role=a.role, kv_events_port=a.kv_events_port,
                        topic=f"kv@{os.environ.get('POD_IP', '127.0.0.1')}:{a.port}@{a.model}", max_lora=a.max_lora)
        while True:
            await asyncio.sleep(3600)

    asyncio.run(run())


if __name__ == "__main__":
    main()
