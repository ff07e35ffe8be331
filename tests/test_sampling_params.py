"""OpenAI / vLLM sampling parameters beyond temperature / top-k / top-p:
presence, frequency and repetition penalties, logit_bias, min_p (engine
model_runner._penalize, numpy reference), their validation, and ``n`` choices
through the API server (non-streaming and streaming)."""
import asyncio
import json
import types

import aiohttp
import numpy as np
import pytest
import torch
from aiohttp import web

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.model_runner import ModelRunner
from llmd_amd.engine.request import SamplingParams
from llmd_amd.serving.api_server import build_server


def _req(prompt, out, **kw):
    return types.SimpleNamespace(params=SamplingParams(**kw), prompt_token_ids=prompt, output_token_ids=out)


def test_penalties_match_numpy_reference():
    V = 32
    rng = np.random.default_rng(0)
    logits = rng.normal(size=(4, V)).astype(np.float32) * 3
    reqs = [_req([1, 2, 3], [5, 5, 7], presence_penalty=0.5, frequency_penalty=0.25),
            _req([4, 4, 9], [9, 10], repetition_penalty=1.3),
            _req([0], [], logit_bias={3: 5.0, 11: -100.0}),
            _req([0], [1], temperature=0.0)]  # untouched row
    got = ModelRunner._penalize(None, torch.from_numpy(logits.copy()), reqs).numpy()
    want = logits.copy()
    for t, c in ((5, 2), (7, 1)):
        want[0, t] -= 0.25 * c + 0.5
    for t in (4, 9, 10):
        want[1, t] = want[1, t] / 1.3 if want[1, t] > 0 else want[1, t] * 1.3
    want[2, 3] += 5.0
    want[2, 11] -= 100.0
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-6)


def test_min_p_masks_low_probability_tokens():
    logits = torch.tensor([[4.0, 3.0, 0.0, -2.0]])
    out = ModelRunner._penalize(None, logits.clone(), [_req([0], [], min_p=0.2, temperature=1.0)])
    p = torch.softmax(logits, -1)[0]
    keep = p >= 0.2 * p.max()
    assert torch.isinf(out[0][~keep]).all() and torch.equal(out[0][keep], logits[0][keep])


@pytest.mark.parametrize("body", [{"presence_penalty": 3}, {"frequency_penalty": -2.5}, {"repetition_penalty": 0},
                                  {"min_p": 1.5}, {"n": 0}, {"top_p": 0}, {"temperature": -1},
                                  {"logit_bias": {"-1": 1.0}}, {"logit_bias": {"5": 101.0}},
                                  {"logit_bias": {"5": float("nan")}}, {"logit_bias": {"32000": 1.0}}])
def test_validation(body):
    with pytest.raises(ValueError):
        SamplingParams.from_openai(body, vocab_size=32000)


def _cfg():
    return EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=128,
                               max_num_batched_tokens=128, max_num_seqs=8, max_model_len=512, enforce_eager=True)


async def _serve(app):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def test_api_n_choices_bias_and_penalties():
    async def main():
        srv = build_server(_cfg())
        r1, port = await _serve(srv.app())
        base = f"http://127.0.0.1:{port}/v1/completions"
        out = {}
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(base, json={"prompt": [5, 6, 7], "max_tokens": 6, "n": 3, "temperature": 1.0,
                                              "seed": 1, "ignore_eos": True, "return_token_ids": True}) as r:
                    out["n"] = await r.json()
                async with s.post(base, json={"prompt": [5, 6, 7], "max_tokens": 5, "temperature": 0,
                                              "logit_bias": {"42": 100}, "return_token_ids": True,
                                              "ignore_eos": True}) as r:
                    out["bias"] = await r.json()
                async with s.post(base, json={"prompt": [5, 6, 7], "max_tokens": 8, "temperature": 0,
                                              "return_token_ids": True, "ignore_eos": True}) as r:
                    out["greedy"] = await r.json()
                async with s.post(base, json={"prompt": [5, 6, 7], "max_tokens": 8, "temperature": 0,
                                              "frequency_penalty": 2.0, "presence_penalty": 2.0,
                                              "return_token_ids": True, "ignore_eos": True}) as r:
                    out["pen"] = await r.json()
                async with s.post(base, json={"prompt": [5, 6, 7], "max_tokens": 4, "n": 2, "stream": True,
                                              "ignore_eos": True, "stream_options": {"include_usage": True}}) as r:
                    out["stream"] = [json.loads(l[5:]) for l in (await r.text()).splitlines()
                                     if l.startswith("data:") and "[DONE]" not in l]
                async with s.post(base, json={"prompt": [5], "presence_penalty": 9}) as r:
                    out["bad"] = r.status
                # a bias key outside the vocabulary would index past the logits row on the device
                async with s.post(base, json={"prompt": [5], "logit_bias": {"10000000": 5}}) as r:
                    out["bad_bias"] = r.status
                async with s.post(base.replace("completions", "chat/completions"),
                                  json={"messages": [{"role": "user", "content": "hi"}],
                                        "logit_bias": {"-3": 5}}) as r:
                    out["bad_bias_chat"] = r.status
            return out
        finally:
            await r1.cleanup()
            srv.aeng.shutdown()

    out = asyncio.run(main())
    ch = out["n"]["choices"]
    assert [c["index"] for c in ch] == [0, 1, 2] and all(len(c["token_ids"]) == 6 for c in ch)
    assert len({tuple(c["token_ids"]) for c in ch}) > 1          # independent samples
    assert out["n"]["usage"] == {"prompt_tokens": 3, "completion_tokens": 18, "total_tokens": 21}
    assert out["bias"]["choices"][0]["token_ids"] == [42] * 5
    g, p = out["greedy"]["choices"][0]["token_ids"], out["pen"]["choices"][0]["token_ids"]
    assert max(np.bincount(p)) <= max(np.bincount(g))            # penalties discourage repeats
    assert len(set(p)) >= len(set(g))
    chunks = [c for c in out["stream"] if c["choices"]]
    per = {0: 0, 1: 0}
    for c in chunks:
        per[c["choices"][0]["index"]] += 1
    assert per[0] >= 1 and per[1] >= 1
    assert out["stream"][-1]["usage"]["completion_tokens"] == 8
    assert out["bad"] == 400
    assert out["bad_bias"] == 400 and out["bad_bias_chat"] == 400
