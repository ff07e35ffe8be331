"""Multimodal serving and encoder disaggregation on CPU:
vision tower token accounting, image placeholders across chunked-prefill
boundaries, image-aware prefix caching, and E/PD over HTTP - a PD server that
pulls embeddings from an encode worker named in `x-encoder-hosts-ports`
produces the same tokens as an aggregated E+PD server."""
import asyncio
import base64
import io

import aiohttp
import torch
from aiohttp import web

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams
from llmd_amd.models.vision import MMInput, VisionConfig, mm_hash, num_image_tokens, smart_resize


def _png(w, h, seed=0):
    from PIL import Image

    g = torch.Generator().manual_seed(seed)
    arr = (torch.rand(h, w, 3, generator=g) * 255).to(torch.uint8).numpy()
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return buf.getvalue()


def _url(b):
    return "data:image/png;base64," + base64.b64encode(b).decode()


def _cfg(**kw):
    base = dict(device="cpu", block_size=16, num_gpu_blocks=128, max_num_batched_tokens=256, max_num_seqs=4,
                max_model_len=1024, enforce_eager=True, seed=0)
    base.update(kw)
    return EngineConfig.create("tiny-vl", **base)


def test_token_accounting():
    v = VisionConfig(max_pixels=16 * 28 * 28, min_pixels=4 * 28 * 28)
    assert smart_resize(56, 84, v) == (56, 84)
    assert num_image_tokens(56, 84, v) == 6
    assert num_image_tokens(1000, 1000, v) <= 16     # capped by max_pixels
    assert num_image_tokens(10, 10, v) >= 4          # raised to min_pixels


def _mm_request(eng, img, text_ids):
    emb = eng.runner.model.encode_image(img)
    n = emb.shape[0]
    tid = eng.cfg.model_config.image_token_id
    ids = text_ids[:5] + [tid] * n + text_ids[5:]
    return ids, [MMInput(offset=5, length=n, mm_hash=mm_hash(img), embeds=emb)]


def test_chunked_prefill_over_image_matches_single_chunk():
    img = _png(84, 112, seed=1)
    text = list(range(10, 40))
    outs = []
    for mbt in (256, 16):  # 16 = the image spans several prefill chunks
        eng = LLMEngine(_cfg(max_num_batched_tokens=mbt, enable_prefix_caching=False))
        ids, mm = _mm_request(eng, img, text)
        r = eng.add_request("a", ids, SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True),
                            mm_inputs=mm)
        while eng.has_unfinished():
            eng.step()
        outs.append(r.output_token_ids)
    assert outs[0] == outs[1]
    # the image matters: a different image changes the continuation's logits path
    eng = LLMEngine(_cfg())
    ids, mm = _mm_request(eng, _png(84, 112, seed=2), text)
    assert len(ids) == len(_mm_request(eng, img, text)[0])


def test_prefix_cache_keys_include_image():
    eng = LLMEngine(_cfg())
    text = list(range(10, 80))
    sp = SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True)
    a, b = _png(56, 56, seed=3), _png(56, 56, seed=4)
    ids, mm = _mm_request(eng, a, text)
    eng.add_request("warm", ids, sp, mm_inputs=mm)
    while eng.has_unfinished():
        eng.step()
    r1 = eng.add_request("same", ids, sp, mm_inputs=_mm_request(eng, a, text)[1])
    ids_b, mm_b = _mm_request(eng, b, text)
    r2 = eng.add_request("other", ids_b, sp, mm_inputs=mm_b)
    while eng.has_unfinished():
        eng.step()
    assert r1.num_cached_tokens > 0      # same image -> prefix hit
    assert r2.num_cached_tokens == 0     # same token ids, different image -> no false hit


async def _serve(app):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def test_epd_over_http_matches_aggregated():
    from llmd_amd.serving.api_server import build_server

    img = _png(84, 56, seed=5)
    body = {"model": "tiny-vl", "max_tokens": 6, "temperature": 0.0, "ignore_eos": True,
            "messages": [{"role": "user", "content": [{"type": "text", "text": "describe"},
                                                      {"type": "image_url", "image_url": {"url": _url(img)}},
                                                      {"type": "text", "text": "briefly"}]}]}

    async def main():
        agg = build_server(_cfg())
        enc = build_server(_cfg())
        pd = build_server(_cfg())
        runners = []
        try:
            ra, pa = await _serve(agg.app())
            re_, pe = await _serve(enc.app())
            rp, pp = await _serve(pd.app())
            runners = [ra, re_, rp]
            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{pa}/v1/chat/completions", json=body) as r:
                    assert r.status == 200, await r.text()
                    want = await r.json()
                async with s.post(f"http://127.0.0.1:{pp}/v1/chat/completions", json=body,
                                  headers={"x-encoder-hosts-ports": f"127.0.0.1:{pe}"}) as r:
                    assert r.status == 200, await r.text()
                    got = await r.json()
                async with s.post(f"http://127.0.0.1:{pe}/v1/encode", json={"images": [_url(img)]}) as r:
                    info = (await r.json())["data"][0]
                async with s.get(f"http://127.0.0.1:{pp}/metrics") as r:
                    metrics = await r.text()
            return want, got, info, metrics
        finally:
            for r in runners:
                await r.cleanup()
            await pd.mm.close()
            for s in (agg, enc, pd):
                s.aeng.shutdown()

    want, got, info, metrics = asyncio.run(main())
    assert got["choices"][0]["message"]["content"] == want["choices"][0]["message"]["content"]
    assert got["usage"]["prompt_tokens"] == want["usage"]["prompt_tokens"]
    assert info["num_tokens"] == num_image_tokens(84, 56, VisionConfig(max_pixels=16 * 28 * 28,
                                                                       min_pixels=4 * 28 * 28))
    assert 'llmd:ec_remote_fetches_total{model_name="tiny-vl"} 1' in metrics
    assert 'llmd:ec_local_encodes_total{model_name="tiny-vl"} 0' in metrics
