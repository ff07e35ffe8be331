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
