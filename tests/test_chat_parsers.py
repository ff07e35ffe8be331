"""Chat templates, reasoning / tool-call parsers and the vLLM flag surface of
the API server (serving/chat_template.py, serving/parsers.py;
agentic-serving and gpt-oss guides: --enable-auto-tool-choice
--tool-call-parser, --reasoning-parser)."""
import argparse
import asyncio
import json
import types

import aiohttp
import pytest
from aiohttp import web

from llmd_amd.engine.config import EngineConfig, add_engine_args, engine_config_from_args
from llmd_amd.serving.api_server import (ServingOptions, add_serving_args, build_server,
                                         serving_options_from_args)
from llmd_amd.serving.chat_template import BUILTIN, ChatTemplate
from llmd_amd.serving.parsers import ChatOutputParser

HARMONY = ("<|channel|>analysis<|message|>User wants weather. Call tool.<|end|>"
           "<|start|>assistant<|channel|>commentary to=functions.get_weather <|constrain|>json"
           "<|message|>{\"city\": \"Paris\"}<|call|>")
HARMONY_FINAL = "<|channel|>analysis<|message|>easy<|end|><|start|>assistant<|channel|>final<|message|>It is 4.<|return|>"


@pytest.mark.parametrize("reasoning,tools,text,want", [
    ("deepseek_r1", None, "let me think</think>\n\nThe answer is 4.", ("let me think", "The answer is 4.", [])),
    ("qwen3", None, "<think>hmm</think>Four.", ("hmm", "Four.", [])),
    ("qwen3", None, "No thinking here.", (None, "No thinking here.", [])),
    (None, "hermes", 'Sure.\n<tool_call>\n{"name": "get_weather", "arguments": {"city": "Paris"}}\n</tool_call>',
     (None, "Sure.", [("get_weather", {"city": "Paris"})])),
    (None, "hermes", "<tool_call>{\"name\": \"a\", \"arguments\": {}}</tool_call><tool_call>{\"name\": \"b\", "
                     "\"arguments\": {\"x\": 1}}</tool_call>", (None, None, [("a", {}), ("b", {"x": 1})])),
    (None, "llama3_json", '<|python_tag|>{"name": "search", "parameters": {"q": "mi355x"}}',
     (None, None, [("search", {"q": "mi355x"})])),
    (None, "llama3_json", "plain answer", (None, "plain answer", [])),
    (None, "mistral", 'ok [TOOL_CALLS] [{"name": "f", "arguments": {"a": 2}}]', (None, "ok", [("f", {"a": 2})])),
    (None, "pythonic", '[get_weather(city="SF"), add(x=1, y=2)]',
     (None, None, [("get_weather", {"city": "SF"}), ("add", {"x": 1, "y": 2})])),
    ("openai_gptoss", "openai", HARMONY, ("User wants weather. Call tool.", None, [("get_weather", {"city": "Paris"})])),
    ("openai_gptoss", "openai", HARMONY_FINAL, ("easy", "It is 4.", [])),
    ("qwen3", "hermes", '<think>need a tool</think><tool_call>{"name": "t", "arguments": {"k": "v"}}</tool_call>',
     ("need a tool", None, [("t", {"k": "v"})])),
])
def test_parsers_extract(reasoning, tools, text, want):
    r, c, calls = ChatOutputParser(reasoning, tools).extract(text)
    assert (r, c) == want[:2]
    assert [(x["function"]["name"], json.loads(x["function"]["arguments"])) for x in calls] == want[2]
    assert all(x["type"] == "function" and x["id"].startswith("chatcmpl-tool-") for x in calls)


@pytest.mark.parametrize("reasoning,tools,text", [
    ("qwen3", "hermes", '<think>step one, step two</think>Hello there.<tool_call>{"name": "t", "arguments": '
                        '{"k": "v"}}</tool_call>'),
    ("deepseek_r1", None, "a b c d</think>\n\nfinal words here"),
    ("openai_gptoss", "openai", HARMONY),
    ("openai_gptoss", "openai", HARMONY_FINAL),
    (None, "llama3_json", '{"name": "search", "parameters": {"q": "x"}}'),
])
def test_streaming_matches_one_shot(reasoning, tools, text):
    """Feeding the text in arbitrary chunks yields the same reasoning /
    content / tool calls as the one-shot parse, and no marker leaks."""
    p = ChatOutputParser(reasoning, tools)
    r0, c0, calls0 = p.extract(text)
    for step in (1, 3, 7):
        st = p.streamer()
        deltas = []
        for k in range(step, len(text) + step, step):
            deltas += st.feed(text[:k])
        tail, called = st.finish()
        deltas += tail
        r = "".join(d.get("reasoning_content", "") for d in deltas)
        c = "".join(d.get("content", "") for d in deltas)
        calls = [tc for d in deltas for tc in d.get("tool_calls", [])]
        assert r == (r0 or "") and c == (c0 or "")
        assert [x["function"]["name"] for x in calls] == [x["function"]["name"] for x in calls0]
        assert called == bool(calls0)
        assert "<think>" not in c and "<tool_call>" not in c and "<|channel|>" not in c


def test_builtin_templates_render_tools_and_round_trip():
    tools = [{"type": "function", "function": {"name": "get_weather", "description": "weather",
                                                "parameters": {"type": "object", "properties": {"city": {}}}}}]
    msgs = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "weather in Paris?"},
            {"role": "assistant", "content": "", "tool_calls": [
                {"id": "c1", "type": "function", "function": {"name": "get_weather",
                                                              "arguments": "{\"city\": \"Paris\"}"}}]},
            {"role": "tool", "tool_call_id": "c1", "content": "sunny"}]
    for style, marks in (("llama3", ["Environment: ipython", "<|python_tag|>", "ipython<|end_header_id|>"]),
                         ("chatml", ["<tools>", "<tool_call>", "<tool_response>"]),
                         ("harmony", ["namespace functions", "to=functions.get_weather", "functions.get_weather to=assistant"]),
                         ("deepseek", ["## Tools", "<｜tool▁call▁begin｜>", "<｜tool▁output▁begin｜>"])):
        out = BUILTIN[style](msgs, True, tools)
        for m in marks:
            assert m in out, (style, m)
        assert "get_weather" in out and "sunny" in out
    # no tools: the plain templates of earlier rounds
    assert BUILTIN["llama3"]([{"role": "user", "content": "hi"}], True, None) == \
        "<|begin_of_text|><|start_header_id|>user<|end_header_id|>\n\nhi<|eot_id|>" \
        "<|start_header_id|>assistant<|end_header_id|>\n\n"


def test_jinja_template_from_tokenizer_config(tmp_path):
    tpl = ("{{ bos_token }}{% for m in messages %}[{{ m['role'] }}]{{ m['content'] }}{% endfor %}"
           "{% if tools %}TOOLS={{ tools | map(attribute='function.name') | join(',') }}{% endif %}"
           "{% if add_generation_prompt %}[assistant]{% endif %}")
    (tmp_path / "tokenizer_config.json").write_text(json.dumps({"chat_template": tpl, "bos_token": "<s>"}))
    t = ChatTemplate("chatml", model_dir=str(tmp_path))
    out = t.render([{"role": "user", "content": "hi"}], True,
                   tools=[{"type": "function", "function": {"name": "f"}}])
    assert out == "<s>[user]hiTOOLS=f[assistant]"
    t2 = ChatTemplate("chatml", template="{{ raise_exception('nope') }}")
    with pytest.raises(Exception, match="nope"):
        t2.render([{"role": "user", "content": "x"}])


def test_vllm_flags_parse():
    p = argparse.ArgumentParser()
    add_engine_args(p)
    add_serving_args(p)
    a = p.parse_args(["--model", "tiny-gpt-oss", "--device", "cpu", "--trust-remote-code", "--async-scheduling",
                      "--tokenizer-mode", "auto", "--disable-sliding-window", "--hf-overrides",
                      '{"num_hidden_layers": 2}', "-O", '{"cudagraph_capture_sizes": [1, 2, 4, 16]}',
                      "--enable-auto-tool-choice", "--tool-call-parser", "openai", "--reasoning-parser",
                      "openai_gptoss", "--disable-access-log-for-endpoints=/health,/metrics",
                      "--limit-mm-per-prompt", '{"image": 2}', "--stream-interval", "4",
                      "--data-parallel-hybrid-lb", "--otlp-traces-endpoint", "http://c:4317",
                      "--ec-transfer-config", '{"ec_connector": "ECCPUConnector", "ec_role": "ec_consumer"}'])
    cfg = engine_config_from_args(a)
    assert cfg.model_config.num_hidden_layers == 2 and cfg.model_config.sliding_window == 0
    assert cfg.model_config.layer_types == ["full_attention"] * 2 and cfg.cuda_graph_max_bs == 16
    o = serving_options_from_args(a)
    assert o.tool_call_parser == "openai" and o.stream_interval == 4 and o.limit_mm_per_prompt == {"image": 2}
    a2 = p.parse_args(["--model", "tiny-llama", "-O", '{"cudagraph_mode": "NONE"}'])
    assert engine_config_from_args(a2).enforce_eager
    with pytest.raises(SystemExit):
        serving_options_from_args(p.parse_args(["--enable-auto-tool-choice"]))
    with pytest.raises(ValueError):
        serving_options_from_args(p.parse_args(["--tool-call-parser", "nope"]))
    with pytest.raises(ValueError):
        engine_config_from_args(p.parse_args(["--hf-overrides", '{"no_such_field": 1}']))


def _cfg():
    return EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                               max_num_batched_tokens=128, max_num_seqs=4, max_model_len=512, enforce_eager=True)


async def _serve(app):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def _scripted(srv, text):
    """Make the engine 'generate' exactly ``text`` (token by token)."""
    ids = srv.tok.encode(text)

    async def gen(rid, prompt, params, *a, **k):
        for i, t in enumerate(ids):
            fin = i == len(ids) - 1
            yield types.SimpleNamespace(new_token_ids=[t], new_logprobs=[0.0], finished=fin,
                                        finish_reason="stop" if fin else None, kv_transfer_params=None)
    srv.aeng.generate = gen


def test_http_tool_calls_and_reasoning():
    text = '<think>I should call it</think><tool_call>{"name": "get_weather", "arguments": {"city": "Paris"}}' \
           '</tool_call>'
    tools = [{"type": "function", "function": {"name": "get_weather", "parameters": {}}}]
    chat = {"model": "tiny-llama", "messages": [{"role": "user", "content": "weather?"}], "tools": tools}

    async def main():
        srv = build_server(_cfg(), opts=ServingOptions(enable_auto_tool_choice=True, tool_call_parser="hermes",
                                                       reasoning_parser="qwen3", stream_interval=3))
        plain = build_server(_cfg())
        _scripted(srv, text)
        r1, port = await _serve(srv.app())
        r2, port2 = await _serve(plain.app())
        out = {}
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions", json=chat) as r:
                    out["full"] = await r.json()
                async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions", json=dict(chat, stream=True)) as r:
                    out["chunks"] = [json.loads(l[5:]) for l in (await r.text()).splitlines()
                                     if l.startswith("data:") and "[DONE]" not in l]
                async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions",
                                  json=dict(chat, tool_choice="none")) as r:
                    out["none"] = await r.json()
                async with s.post(f"http://127.0.0.1:{port2}/v1/chat/completions",
                                  json=dict(chat, tool_choice="auto")) as r:
                    out["auto_disabled"] = (r.status, await r.json())
                async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions/render", json=chat) as r:
                    rendered_tools = await r.json()
                async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions/render",
                                  json=dict(chat, tool_choice="none")) as r:
                    rendered_none = await r.json()
            out["render"] = (len(rendered_tools["token_ids"]), len(rendered_none["token_ids"]))
            return out
        finally:
            await r1.cleanup()
            await r2.cleanup()
            srv.aeng.shutdown()
            plain.aeng.shutdown()

    out = asyncio.run(main())
    ch = out["full"]["choices"][0]
    assert ch["finish_reason"] == "tool_calls"
    assert ch["message"]["reasoning_content"] == "I should call it" and ch["message"]["content"] is None
    tc = ch["message"]["tool_calls"][0]
    assert tc["function"]["name"] == "get_weather" and json.loads(tc["function"]["arguments"]) == {"city": "Paris"}
    deltas = [c["choices"][0]["delta"] for c in out["chunks"] if c.get("choices")]
    assert "".join(d.get("reasoning_content", "") for d in deltas) == "I should call it"
    assert "".join(d.get("content", "") for d in deltas) == ""
    calls = [t for d in deltas for t in d.get("tool_calls", [])]
    assert [t["function"]["name"] for t in calls] == ["get_weather"] and calls[0]["index"] == 0
    assert out["chunks"][-1]["choices"][0]["finish_reason"] == "tool_calls"
    # tool_choice none: the tools stay out of the prompt and the reply is not parsed for calls
    assert out["none"]["choices"][0]["message"]["tool_calls"] == []
    assert out["auto_disabled"][0] == 400 and "enable-auto-tool-choice" in out["auto_disabled"][1]["error"]["message"]
    assert out["render"][0] > out["render"][1]  # the tool block is rendered into the prompt
