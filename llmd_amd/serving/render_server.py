"""Standalone tokenizer / render sidecar (reference
docs/architecture/advanced/kv-management/kv-indexer.md:104-113 `vllm launch
render`, prefix-cache-aware-routing.md:46).

A CPU-only process that serves the exact token ids a model server would
compute - no weights, no GPU - so the router's ``token-producer`` (and
the precise prefix-cache producer) can run next to the EPP instead of asking
a loaded engine. Same wire format as the engine's endpoints:

  POST /v1/completions/render       {"prompt": str|[str]|[int]} -> token_ids
  POST /v1/chat/completions/render  {"messages": [...]}         -> token_ids
  POST /tokenize, /detokenize
  GET  /health, /v1/models

  python -m llmd_amd.serving.render_server --model llama-3-8b [--tokenizer DIR] --port 8300
"""
from __future__ import annotations

import argparse
import logging

from aiohttp import web

from llmd_amd.engine.config import get_model_config

from .chat_template import ChatTemplate, render_tools, style_for
from .tokenizer import load_tokenizer

log = logging.getLogger("llmd.render")


class RenderServer:
    def __init__(self, model: str, tokenizer: str | None = None, served_name: str | None = None,
                 max_model_len: int = 32768, chat_template: str | None = None, enable_auto_tool_choice: bool = False):
        mc = get_model_config(model)
        self.mc = mc
        self.name = served_name or model
        self.max_model_len = max_model_len
        self.tok = load_tokenizer(tokenizer, mc.vocab_size, mc.bos_token_id, mc.eos_ids[0])
        self.template = ChatTemplate(style_for(mc.model_type), model_dir=tokenizer, template=chat_template)
        self.auto_tools = enable_auto_tool_choice
        self.n = 0

    def app(self) -> web.Application:
        app = web.Application(client_max_size=64 * 1024 * 1024)
        r = app.router
        r.add_get("/health", self.health)
        r.add_get("/v1/models", self.models)
        r.add_post("/v1/completions/render", self.render_completion)
        r.add_post("/v1/chat/completions/render", self.render_chat)
        r.add_post("/tokenize", self.tokenize)
        r.add_post("/detokenize", self.detokenize)
        return app

    async def health(self, req):
        return web.Response(text="")

    async def models(self, req):
        return web.json_response({"object": "list", "data": [{"id": self.name, "object": "model",
                                                             "owned_by": "llmd-amd", "root": self.name}]})

    def _prompt(self, p):
        if isinstance(p, str):
            return self.tok.encode(p)
        if isinstance(p, list) and p and isinstance(p[0], int):
            return list(p)
        if isinstance(p, list) and p and isinstance(p[0], str):
            return self.tok.encode(p[0])
        raise ValueError("unsupported prompt format")

    def _resp(self, body, ids):
        self.n += 1
        return web.json_response({"model": body.get("model") or self.name, "token_ids": ids,
                                  "prompt_token_ids": ids, "count": len(ids), "max_model_len": self.max_model_len})

    async def render_completion(self, req):
        body = await req.json()
        try:
            ids = self._prompt(body.get("prompt"))
        except ValueError as e:
            return web.json_response({"error": {"message": str(e), "code": 400}}, status=400)
        return self._resp(body, ids)

    async def render_chat(self, req):
        body = await req.json()
        msgs = body.get("messages")
        if not isinstance(msgs, list) or not msgs:
            return web.json_response({"error": {"message": "messages is required", "code": 400}}, status=400)
        ids = self.tok.encode(self.template.render(msgs, body.get("add_generation_prompt", True),
                                                   tools=render_tools(body, self.auto_tools)))
        return self._resp(body, ids)

    async def tokenize(self, req):
        body = await req.json()
        if "messages" in body:
            ids = self.tok.encode(self.template.render(body["messages"], body.get("add_generation_prompt", True),
                                                       tools=render_tools(body, self.auto_tools)))
        else:
            ids = self._prompt(body.get("prompt", ""))
        return web.json_response({"tokens": ids, "count": len(ids), "max_model_len": self.max_model_len})

    async def detokenize(self, req):
        body = await req.json()
        return web.json_response({"prompt": self.tok.decode(body.get("tokens", []))})


def main(argv=None):
    p = argparse.ArgumentParser("llmd-amd render")
    p.add_argument("--model", default="llama-3-8b")
    p.add_argument("--tokenizer", default=None)
    p.add_argument("--served-model-name", default=None)
    p.add_argument("--max-model-len", type=int, default=32768)
    p.add_argument("--chat-template", default=None)
    p.add_argument("--enable-auto-tool-choice", action="store_true",
                   help="render tools when a request omits tool_choice (match the engine's flag)")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8300)
    a = p.parse_args(argv)
    logging.basicConfig(level="INFO")
    srv = RenderServer(a.model, a.tokenizer, a.served_model_name, a.max_model_len, a.chat_template,
                       a.enable_auto_tool_choice)
    web.run_app(srv.app(), host=a.host, port=a.port, access_log=None)


if __name__ == "__main__":
    main()
