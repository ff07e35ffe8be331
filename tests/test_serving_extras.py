"""Standalone render sidecar (C19) == the engine's own render endpoints, and
the resilience (IRO EngineAdapter) endpoints: status / pause / resume /
abort_all / drain."""
import asyncio

import aiohttp
from aiohttp import web

from llmd_amd.engine.config import EngineConfig
from llmd_amd.serving.api_server import build_server
from llmd_amd.serving.render_server import RenderServer


async def _serve(app):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def _cfg():
    return EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                               max_num_batched_tokens=128, max_num_seqs=4, max_model_len=512, enforce_eager=True)


def test_render_server_matches_engine_and_ft_endpoints():
    chat = {"model": "tiny-llama", "messages": [{"role": "user", "content": "hello there"}]}
    comp = {"model": "tiny-llama", "prompt": "the quick brown fox"}

    async def main():
        eng = build_server(_cfg())
        rs = RenderServer("tiny-llama")
        r1, p1 = await _serve(eng.app())
        r2, p2 = await _serve(rs.app())
        try:
            async with aiohttp.ClientSession() as s:
                res = {}
                for port, tag in ((p1, "eng"), (p2, "render")):
                    async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions/render", json=chat) as r:
                        res[tag + "_chat"] = (await r.json())["token_ids"]
                    async with s.post(f"http://127.0.0.1:{port}/v1/completions/render", json=comp) as r:
                        res[tag + "_comp"] = (await r.json())["token_ids"]
                base = f"http://127.0.0.1:{p1}"
                async with s.get(base + "/fault_tolerance/status") as r:
                    res["st0"] = await r.json()
                async with s.post(base + "/fault_tolerance/apply", json={"action": "pause"}) as r:
                    assert r.status == 200
                async with s.get(base + "/fault_tolerance/status") as r:
                    res["st1"] = await r.json()
                async with s.post(base + "/fault_tolerance/apply", json={"action": "resume"}) as r:
                    assert r.status == 200
                async with s.post(base + "/fault_tolerance/apply", json={"action": "explode"}) as r:
                    res["bad"] = r.status
                async with s.post(base + "/v1/completions", json=dict(comp, max_tokens=3)) as r:
                    res["after"] = r.status
            return res
        finally:
            await r1.cleanup()
            await r2.cleanup()
            eng.aeng.shutdown()

    res = asyncio.run(main())
    assert res["eng_chat"] == res["render_chat"] and res["eng_comp"] == res["render_comp"]
    assert res["st0"]["status"] == "healthy" and res["st1"]["status"] == "paused"
    assert res["bad"] == 400 and res["after"] == 200


def test_embeddings_responses_messages_generate_endpoints():
    async def main():
        eng = build_server(_cfg())
        r1, p1 = await _serve(eng.app())
        base = f"http://127.0.0.1:{p1}"
        out = {}
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(base + "/v1/embeddings", json={"model": "tiny-llama",
                                                                 "input": ["hello world", "goodbye"]}) as r:
                    out["emb"] = (r.status, await r.json())
                async with s.post(base + "/v1/responses", json={"model": "tiny-llama", "input": "hi",
                                                                "instructions": "be brief", "max_output_tokens": 4,
                                                                "temperature": 0}) as r:
                    out["resp"] = (r.status, await r.json())
                async with s.post(base + "/v1/messages", json={
                        "model": "tiny-llama", "max_tokens": 3, "system": "sys", "temperature": 0,
                        "messages": [{"role": "user", "content": [{"type": "text", "text": "hello"}]}]}) as r:
                    out["msg"] = (r.status, await r.json())
                async with s.post(base + "/inference/v1/generate", json={
                        "token_ids": [5, 6, 7, 8], "sampling_params": {"max_tokens": 5, "temperature": 0,
                                                                        "ignore_eos": True}}) as r:
                    out["gen"] = (r.status, await r.json())
                async with s.post(base + "/v1/completions", json={"model": "tiny-llama", "prompt": [5, 6, 7, 8],
                                                                  "max_tokens": 5, "temperature": 0,
                                                                  "ignore_eos": True,
                                                                  "return_token_ids": True}) as r:
                    out["cmp"] = (r.status, await r.json())
        finally:
            await r1.cleanup()
            eng.aeng.shutdown()
        return out

    out = asyncio.run(main())
    st, emb = out["emb"]
    assert st == 200 and len(emb["data"]) == 2
    v = emb["data"][0]["embedding"]
    assert len(v) == 256 and abs(sum(x * x for x in v) - 1.0) < 1e-3
    assert emb["data"][0]["embedding"] != emb["data"][1]["embedding"]
    st, resp = out["resp"]
    assert st == 200 and resp["object"] == "response" and resp["usage"]["output_tokens"] == 4
    assert resp["output"][0]["content"][0]["type"] == "output_text"
    st, msg = out["msg"]
    assert st == 200 and msg["type"] == "message" and msg["stop_reason"] == "max_tokens"
    assert msg["usage"]["output_tokens"] == 3
    st, gen = out["gen"]
    assert st == 200 and len(gen["choices"][0]["token_ids"]) == 5
    assert gen["choices"][0]["token_ids"] == out["cmp"][1]["choices"][0]["token_ids"]


def test_out_of_vocab_token_ids_rejected_engine_survives():
    """Token-id prompts outside the vocabulary get a 400 instead of reaching
    the embedding gather (which would take the engine loop down)."""
    async def main():
        eng = build_server(_cfg())
        r1, port = await _serve(eng.app())
        base = f"http://127.0.0.1:{port}"
        v = eng.cfg.model_config.vocab_size
        try:
            async with aiohttp.ClientSession() as s:
                out = {}
                for tag, body, path in (
                        ("comp", {"prompt": [1, 2, v + 5], "max_tokens": 2}, "/v1/completions"),
                        ("batch", {"prompt": [[1, 2], [3, -1]], "max_tokens": 2}, "/v1/completions"),
                        ("float", {"prompt": [1, 2.5], "max_tokens": 2}, "/v1/completions"),
                        ("gen", {"token_ids": [v], "sampling_params": {"max_tokens": 2}}, "/inference/v1/generate"),
                        ("ok", {"prompt": [1, 2, v - 1], "max_tokens": 2}, "/v1/completions")):
                    async with s.post(base + path, json=dict(body, model="tiny-llama")) as r:
                        out[tag] = (r.status, await r.json())
            return out, eng.aeng.dead
        finally:
            await r1.cleanup()
            eng.aeng.shutdown()

    out, dead = asyncio.run(main())
    for tag in ("comp", "batch", "float", "gen"):
        assert out[tag][0] == 400, (tag, out[tag])
    assert "out of vocabulary" in out["comp"][1]["error"]["message"]
    assert out["ok"][0] == 200 and out["ok"][1]["usage"]["completion_tokens"] == 2
    assert dead is None


def test_messages_streaming_event_sequence():
    """Anthropic /v1/messages with stream=true: message_start, content_block_start,
    deltas, content_block_stop, message_delta (stop_reason, usage), message_stop;
    the concatenated deltas equal the non-streaming answer."""
    body = {"model": "tiny-llama", "max_tokens": 6, "temperature": 0, "system": "s",
            "messages": [{"role": "user", "content": "hello there"}]}

    async def main():
        eng = build_server(_cfg())
        r1, p1 = await _serve(eng.app())
        base = f"http://127.0.0.1:{p1}/v1/messages"
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(base, json=body) as r:
                    full = await r.json()
                async with s.post(base, json=dict(body, stream=True)) as r:
                    ctype = r.headers.get("Content-Type", "")
                    raw = await r.text()
        finally:
            await r1.cleanup()
            eng.aeng.shutdown()
        return full, ctype, raw

    import json

    full, ctype, raw = asyncio.run(main())
    assert ctype.startswith("text/event-stream")
    events = []
    for block in raw.strip().split("\n\n"):
        lines = dict(l.split(": ", 1) for l in block.splitlines() if ": " in l)
        events.append((lines["event"], json.loads(lines["data"])))
    names = [e for e, _ in events]
    assert names[0] == "message_start" and names[1] == "content_block_start"
    assert names[-3:] == ["content_block_stop", "message_delta", "message_stop"]
    text = "".join(d["delta"]["text"] for e, d in events if e == "content_block_delta")
    assert text == full["content"][0]["text"]
    md = dict(events)["message_delta"]
    assert md["delta"]["stop_reason"] == full["stop_reason"] == "max_tokens"
    assert md["usage"]["output_tokens"] == full["usage"]["output_tokens"] == 6
    assert dict(events)["message_start"]["message"]["usage"]["input_tokens"] == full["usage"]["input_tokens"]
