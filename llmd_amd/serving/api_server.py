"""OpenAI-compatible HTTP server for the llmd_amd engine.

Endpoints
  GET  /health                     liveness (returns immediately)
  GET  /v1/models                  readiness (model loaded) + LoRA adapters
  GET  /metrics                    Prometheus, vLLM-compatible names
  POST /v1/completions             (stream / non-stream, kv_transfer_params)
  POST /v1/chat/completions        (text + image parts)
  POST /v1/embeddings, /v1/responses, /v1/messages (Anthropic),
       /inference/v1/generate (token in / token out) - the request surfaces
       the router's openai-parser knows (docs/api-reference/epp-http-apis.md)
  POST /v1/completions/render      exact token ids (router token-producer)
  POST /v1/chat/completions/render
  POST /tokenize, /detokenize
  POST /pause, /resume, /reset_prefix_cache   (IRO-ready lifecycle hooks)
  GET  /is_paused
  POST /init_weight_update_group, /update_weights, /update_weights_from_disk,
       /destroy_weight_update_group, /sleep, /wake_up; GET /is_sleeping
       (RL rollout weight sync + engine sleep, SURVEY M17, engine/weight_sync.py)
  GET  /fault_tolerance/status, POST /fault_tolerance/apply   (Inference
       Resilience Operator EngineAdapter contract, proposals/
       inference-resilience-operator.md:66-256; faults are also published as
       ``vllm_fault`` events on the KV-event channel when it is enabled)
P/D: a body with ``kv_transfer_params.do_remote_decode`` makes this engine a
prefill producer (the response carries the params the decoder needs);
``do_remote_prefill`` makes it pull KV over kvx before decoding.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import time
import uuid
from dataclasses import dataclass
from typing import Optional

from aiohttp import web

from llmd_amd.engine.config import EngineConfig, add_engine_args, engine_config_from_args
from llmd_amd.engine.request import SamplingParams

from .async_engine import AsyncEngine, EngineDeadError
from .chat_template import ChatTemplate, render_tools, style_for
from .parsers import ChatOutputParser
from .tokenizer import load_tokenizer

log = logging.getLogger("llmd.api")


def _err(status: int, msg: str, typ: str = "invalid_request_error"):
    return web.json_response({"error": {"message": msg, "type": typ, "code": status}}, status=status)


@dataclass
class ServingOptions:
    """Front-end options (vLLM flag names): chat template, output parsers,
    streaming granularity, multimodal limits / roles."""
    chat_template: Optional[str] = None
    enable_auto_tool_choice: bool = False
    tool_call_parser: Optional[str] = None
    reasoning_parser: Optional[str] = None
    stream_interval: int = 1
    limit_mm_per_prompt: Optional[dict] = None
    mm_encoder_only: bool = False


class OpenAIServer:
    def __init__(self, aeng: AsyncEngine, cfg: EngineConfig, tokenizer=None, lora_manager=None,
                 opts: Optional[ServingOptions] = None):
        self.aeng = aeng
        self.cfg = cfg
        self.name = cfg.served_name
        mc = cfg.model_config
        self.tok = tokenizer or load_tokenizer(cfg.tokenizer, mc.vocab_size, mc.bos_token_id, mc.eos_ids[0])
        self._vocab = mc.vocab_size
        self.lora = lora_manager
        self.opts = opts or ServingOptions()
        self.template = ChatTemplate(style_for(mc.model_type), model_dir=cfg.tokenizer,
                                     template=self.opts.chat_template)
        self.parser = (ChatOutputParser(self.opts.reasoning_parser, self.opts.tool_call_parser)
                       if self.opts.reasoning_parser or self.opts.tool_call_parser else None)
        self.ready = True
        self.extra_metrics = []  # callables returning bytes
        self.mm = None
        if mc.vision_config is not None:  # multimodal model: image parts, EC connector, encode role
            from .multimodal import MultimodalFrontend

            self.mm = MultimodalFrontend(aeng, cfg, self.tok)
            self.extra_metrics.append(lambda: self.mm.metrics_text().encode())

    # ------------------------------------------------------------ app
    def app(self) -> web.Application:
        app = web.Application(client_max_size=256 * 1024 * 1024)
        r = app.router
        r.add_get("/health", self.health)
        r.add_get("/v1/models", self.models)
        r.add_get("/metrics", self.metrics)
        r.add_post("/v1/completions", self.completions)
        r.add_post("/v1/chat/completions", self.chat)
        r.add_post("/v1/completions/render", self.render_completion)
        r.add_post("/v1/chat/completions/render", self.render_chat)
        r.add_post("/tokenize", self.tokenize)
        r.add_post("/detokenize", self.detokenize)
        r.add_post("/pause", self.pause)
        r.add_post("/resume", self.resume)
        r.add_get("/is_paused", self.is_paused)
        r.add_post("/reset_prefix_cache", self.reset_prefix_cache)
        r.add_post("/init_weight_update_group", self.init_weight_update_group)
        r.add_post("/update_weights", self.update_weights)
        r.add_post("/update_weights_from_disk", self.update_weights_from_disk)
        r.add_post("/destroy_weight_update_group", self.destroy_weight_update_group)
        r.add_post("/sleep", self.sleep)
        r.add_post("/wake_up", self.wake_up)
        r.add_get("/is_sleeping", self.is_sleeping)
        r.add_get("/fault_tolerance/status", self.ft_status)
        r.add_post("/fault_tolerance/apply", self.ft_apply)
        r.add_post("/v1/embeddings", self.embeddings)
        r.add_post("/v1/responses", self.responses)
        r.add_post("/v1/messages", self.messages)
        r.add_post("/inference/v1/generate", self.generate_tokens)
        r.add_post("/v1/load_lora_adapter", self.load_lora)
        r.add_post("/v1/unload_lora_adapter", self.unload_lora)
        if self.mm is not None:
            r.add_post("/v1/encode", self.mm.http_encode)
            r.add_get("/v1/ec/{mm_hash}", self.mm.http_ec)
        app.on_startup.append(self._start_fault_monitor)
        app.on_cleanup.append(self._stop_fault_monitor)
        return app

    async def health(self, req):
        if self.aeng.dead is not None:
            return web.Response(status=503, text="engine dead")
        return web.Response(text="")

    async def models(self, req):
        data = [{"id": self.name, "object": "model", "created": int(time.time()), "owned_by": "llmd-amd",
                 "root": self.cfg.model, "parent": None, "max_model_len": self.cfg.sched.max_model_len}]
        if self.lora is not None:
            for n in self.lora.names():
                data.append({"id": n, "object": "model", "created": int(time.time()), "owned_by": "llmd-amd",
                             "root": n, "parent": self.name})
        return web.json_response({"object": "list", "data": data})

    async def metrics(self, req):
        body = self.aeng.engine.metrics.render()
        for f in self.extra_metrics:
            body += f()
        return web.Response(body=body, content_type="text/plain", charset="utf-8")

    # ------------------------------------------------------------ helpers
    def _token_ids(self, ids) -> list[int]:
        """Client-supplied token ids: integers inside the vocabulary (an
        out-of-range id would fault the embedding gather inside the step)."""
        v = self.cfg.model_config.vocab_size
        out = []
        for t in ids:
            if isinstance(t, bool) or not isinstance(t, int):
                raise ValueError(f"token ids must be integers, got {t!r}")
            if not 0 <= t < v:
                raise ValueError(f"Token id {t} is out of vocabulary (vocab size {v})")
            out.append(t)
        return out

    def _prompt_ids(self, body) -> list[list[int]]:
        p = body.get("prompt")
        if p is None:
            raise ValueError("prompt is required")
        if isinstance(p, str):
            return [self.tok.encode(p)]
        if isinstance(p, list) and p and isinstance(p[0], int):
            return [self._token_ids(p)]
        if isinstance(p, list) and p and isinstance(p[0], str):
            return [self.tok.encode(x) for x in p]
        if isinstance(p, list) and p and isinstance(p[0], list):
            return [self._token_ids(x) for x in p]
        raise ValueError("unsupported prompt format")

    def _tools_active(self, body) -> bool:
        """OpenAI ``tools`` / ``tool_choice`` semantics (vLLM): ``auto`` needs
        --enable-auto-tool-choice and a --tool-call-parser; ``none`` hides the
        tools from the template; no tool_choice means auto when enabled."""
        tools = body.get("tools")
        if not tools:
            return False
        tc = body.get("tool_choice")
        if tc == "none":
            return False
        enabled = self.opts.enable_auto_tool_choice and self.opts.tool_call_parser
        if tc == "auto" and not enabled:
            raise ValueError('"auto" tool choice requires --enable-auto-tool-choice and --tool-call-parser to be set')
        if tc in ("required",) or isinstance(tc, dict):
            if not self.opts.tool_call_parser:
                raise ValueError("tool_choice 'required' / named functions need --tool-call-parser")
            return True
        return bool(enabled)

    def _chat_ids(self, body) -> list[int]:
        msgs = body.get("messages")
        if not isinstance(msgs, list) or not msgs:
            raise ValueError("messages is required")
        if self.mm is not None and self._has_images(body):
            raise ValueError("image inputs need the async multimodal path")
        self._tools_active(body)  # validates tool_choice
        tools = render_tools(body, bool(self.opts.enable_auto_tool_choice and self.opts.tool_call_parser))
        kw = dict(body.get("chat_template_kwargs") or {})
        return self.tok.encode(self.template.render(msgs, body.get("add_generation_prompt", True), tools=tools,
                                                    **kw))

    @staticmethod
    def _n_images(body) -> int:
        from .multimodal import image_parts

        return len(image_parts(body.get("messages") or []))

    @staticmethod
    def _has_images(body) -> bool:
        from .multimodal import image_parts

        return bool(image_parts(body.get("messages") or []))

    async def _chat_mm(self, body, headers):
        """Chat prompt with image parts -> (token ids with placeholders, MMInputs with embeddings)."""
        from .multimodal import mark_images

        msgs = body.get("messages")
        if not isinstance(msgs, list) or not msgs:
            raise ValueError("messages is required")
        lim = (self.opts.limit_mm_per_prompt or {}).get("image")
        if lim is not None and self._n_images(body) > int(lim):
            raise ValueError(f"At most {lim} image(s) may be provided in one prompt (--limit-mm-per-prompt)")
        text = self.template.render(mark_images(msgs), body.get("add_generation_prompt", True))
        return await self.mm.prepare(body, text, headers)

    def _lora_id(self, body) -> int:
        m = body.get("model")
        if self.lora is not None and m and m != self.name:
            return self.lora.id_of(m)
        return 0

    def _check_model(self, body):
        m = body.get("model")
        if m is None or m == self.name or m == self.cfg.model:
            return None
        if self.lora is not None and self.lora.has(m):
            return None
        return _err(404, f"The model `{m}` does not exist.", "NotFoundError")

    @staticmethod
    def _priority(req, body) -> int:
        if "priority" in body:
            return int(body["priority"])
        return 0

    # ------------------------------------------------------------ completions
    async def completions(self, req: web.Request):
        return await self._serve(req, chat=False)

    async def chat(self, req: web.Request):
        return await self._serve(req, chat=True)

    async def _serve(self, req: web.Request, chat: bool):
        """Engine request span ``llm_request`` (vLLM's name), child of
        the incoming W3C ``traceparent`` (router / sidecar)."""
        from llmd_amd.utils.tracing import span

        with span("llm_request", {"path": req.path, "model": self.name},
                  traceparent=req.headers.get("traceparent")):
            return await self._serve_inner(req, chat)

    async def _serve_inner(self, req: web.Request, chat: bool):
        if self.opts.mm_encoder_only:
            return _err(400, "this instance runs with --mm-encoder-only: it serves /v1/encode, not generation")
        try:
            body = await req.json()
        except Exception:  # noqa: BLE001
            return _err(400, "invalid JSON body")
        bad = self._check_model(body)
        if bad is not None:
            return bad
        mm = None
        try:
            if chat and self.mm is not None and self._has_images(body):
                ids0, mm = await self._chat_mm(body, req.headers)
                prompts = [ids0]
            else:
                prompts = [self._chat_ids(body)] if chat else self._prompt_ids(body)
            tools_on = chat and self._tools_active(body)
            params = SamplingParams.from_openai(body, default_max=16 if not chat else
                                                max(1, self.cfg.sched.max_model_len - 1), vocab_size=self._vocab)
        except (ValueError, TypeError) as e:
            return _err(400, str(e))
        except RuntimeError as e:  # encoder (EC connector) failure
            return _err(502, str(e), "BadGateway")
        for p in prompts:
            if len(p) == 0:
                return _err(400, "empty prompt")
            if len(p) + 1 > self.cfg.sched.max_model_len:
                return _err(400, f"This model's maximum context length is {self.cfg.sched.max_model_len} "
                                 f"tokens. However, you requested {len(p)} tokens in the prompt.")
            if chat:
                params.max_tokens = min(params.max_tokens, self.cfg.sched.max_model_len - len(p))
        ktp = body.get("kv_transfer_params")
        prio = self._priority(req, body)
        lora = self._lora_id(body)
        rid_base = req.headers.get("x-request-id") or f"{'chatcmpl' if chat else 'cmpl'}-{uuid.uuid4().hex}"
        stream = bool(body.get("stream", False))
        include_usage = bool((body.get("stream_options") or {}).get("include_usage", False))
        created = int(time.time())
        model_name = body.get("model") or self.name
        # one engine request per (prompt, sample): choice index = prompt * n + sample; the n
        # samples of a prompt share its prefix blocks through prefix caching
        jobs = [(ids, self._choice_params(params, j)) for ids in prompts for j in range(params.n)]
        rids = [f"{rid_base}-{k}" if len(jobs) > 1 else rid_base for k in range(len(jobs))]
        if stream:
            if len(prompts) > 1:
                return _err(400, "streaming supports a single prompt")
            return await self._stream(req, rids, prompts[0], [pj for _, pj in jobs], prio, ktp, lora, chat,
                                      include_usage, created, model_name, mm, tools_on, rid_base)

        async def one(k, ids, pk):
            text_ids, lps, last = [], [], None
            async for o in self.aeng.generate(rids[k], ids, pk, prio, ktp, lora, mm):
                text_ids.extend(o.new_token_ids)
                lps.extend(o.new_logprobs)
                last = o
                text = self.tok.decode(text_ids)
                if pk.stop and any(s in text for s in pk.stop):
                    self.aeng.abort(rids[k])
                    break
            return ids, text_ids, lps, last
        try:
            results = await asyncio.gather(*[one(k, ids, pk) for k, (ids, pk) in enumerate(jobs)])
        except EngineDeadError as e:
            return _err(503, str(e), "ServiceUnavailable")
        except Exception as e:  # noqa: BLE001
            return _err(500, f"{type(e).__name__}: {e}", "InternalServerError")
        choices, n_prompt, n_out = [], 0, 0
        out_ktp = None
        for i, (ids, toks, lps, last) in enumerate(results):
            text = self.tok.decode(toks)
            finish = last.finish_reason if last is not None else "abort"
            if params.stop:
                for s in params.stop:
                    k = text.find(s)
                    if k >= 0:
                        text, finish = text[:k], "stop"
            if i % params.n == 0:
                n_prompt += len(ids)  # a prompt counts once however many samples it has
            n_out += len(toks)
            if last is not None and last.kv_transfer_params is not None:
                out_ktp = last.kv_transfer_params
            ch = {"index": i, "finish_reason": finish}
            if chat:
                msg = {"role": "assistant", "content": text}
                if self.parser is not None:
                    r, c, calls = self.parser.extract(text, use_tools=tools_on)
                    msg = {"role": "assistant", "content": c, "tool_calls": calls}
                    if self.parser.reasoning is not None:
                        msg["reasoning_content"] = r
                    if calls:
                        ch["finish_reason"] = "tool_calls"
                ch["message"] = msg
            else:
                ch["text"] = text
                if params.logprobs:
                    ch["logprobs"] = {"token_logprobs": lps, "tokens": [self.tok.decode([t]) for t in toks]}
            if body.get("return_token_ids"):
                ch["token_ids"] = toks
            choices.append(ch)
        resp = {"id": rid_base, "object": "chat.completion" if chat else "text_completion", "created": created,
                "model": model_name, "choices": choices,
                "usage": {"prompt_tokens": n_prompt, "completion_tokens": n_out,
                          "total_tokens": n_prompt + n_out}}
        if out_ktp is not None or (ktp and ktp.get("do_remote_decode")):
            resp["kv_transfer_params"] = out_ktp
        return web.json_response(resp)

    @staticmethod
    def _choice_params(params: SamplingParams, j: int) -> SamplingParams:
        """Sample j of an ``n > 1`` request: its own seed stream (seed + j when the
        client fixed one, else a fresh random one per sample)."""
        if params.n == 1:
            return params
        import dataclasses

        return dataclasses.replace(params, seed=(params.seed + j) if params.seed is not None else None)

    async def _stream(self, req, rids, ids, plist, prio, ktp, lora, chat, include_usage, created, model_name,
                      mm=None, tools_on=False, rid=None):
        """SSE stream of one prompt's ``n`` choices (chunks of different choices
        interleave, each tagged with its ``index``)."""
        rid = rid or rids[0]
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream", "Cache-Control": "no-cache"})
        await resp.prepare(req)
        obj = "chat.completion.chunk" if chat else "text_completion"
        wlock = asyncio.Lock()
        n_outs = [0] * len(rids)

        async def send(d):
            async with wlock:
                await resp.write(b"data: " + json.dumps(d).encode() + b"\n\n")

        def chunk(idx, body, finish):
            return {"id": rid, "object": obj, "created": created, "model": model_name,
                    "choices": [dict(body, index=idx, finish_reason=finish)]}

        async def one_choice(idx, crid, params):
            toks: list[int] = []
            sent = ""
            n_emitted = 0
            if chat:
                await send(chunk(idx, {"delta": {"role": "assistant", "content": ""}}, None))
            st = self.parser.streamer(tools_on) if (chat and self.parser is not None) else None
            every = max(1, int(self.opts.stream_interval))
            async for o in self.aeng.generate(crid, ids, params, prio, ktp, lora, mm):
                toks.extend(o.new_token_ids)
                n_outs[idx] = len(toks)
                if not o.finished and len(toks) - n_emitted < every:  # --stream-interval
                    continue
                n_emitted = len(toks)
                text = self.tok.decode(toks)
                stop_hit = False
                if params.stop:
                    for s in params.stop:
                        k = text.find(s)
                        if k >= 0:
                            text, stop_hit = text[:k], True
                delta = text[len(sent):] if text.startswith(sent) else text
                sent = text
                finish = "stop" if stop_hit else (o.finish_reason if o.finished else None)
                if st is not None:  # reasoning / tool-call parsing: parsed deltas, then the final chunk
                    deltas = st.feed(text)
                    if finish is not None:
                        tail, called = st.finish()
                        deltas += tail
                        if called:
                            finish = "tool_calls"
                    for k, dl in enumerate(deltas):
                        await send(chunk(idx, {"delta": dl}, finish if k == len(deltas) - 1 else None))
                    if finish is not None and not deltas:
                        await send(chunk(idx, {"delta": {}}, finish))
                else:
                    d = chunk(idx, {"delta": {"content": delta}} if chat else {"text": delta}, finish)
                    if o.finished and o.kv_transfer_params is not None:
                        d["kv_transfer_params"] = o.kv_transfer_params
                    await send(d)
                if stop_hit:
                    self.aeng.abort(crid)
                    break

        try:
            await asyncio.gather(*[one_choice(i, crid, p) for i, (crid, p) in enumerate(zip(rids, plist))])
        except (ConnectionResetError, asyncio.CancelledError):
            for crid in rids:
                self.aeng.abort(crid)
            raise
        except Exception as e:  # noqa: BLE001
            for crid in rids:
                self.aeng.abort(crid)
            await send({"error": {"message": str(e), "type": type(e).__name__}})
        if include_usage:
            n_out = sum(n_outs)
            await send({"id": rid, "object": obj, "created": created, "model": model_name, "choices": [],
                        "usage": {"prompt_tokens": len(ids), "completion_tokens": n_out,
                                  "total_tokens": len(ids) + n_out}})
        await resp.write(b"data: [DONE]\n\n")
        await resp.write_eof()
        return resp

    # ------------------------------------------------------------ render / tokenize
    async def render_completion(self, req):
        body = await req.json()
        try:
            ids = self._prompt_ids(body)
        except ValueError as e:
            return _err(400, str(e))
        return web.json_response({"model": body.get("model") or self.name, "token_ids": ids[0],
                                  "prompt_token_ids": ids[0], "count": len(ids[0]),
                                  "max_model_len": self.cfg.sched.max_model_len})

    async def render_chat(self, req):
        body = await req.json()
        try:
            ids = self._chat_ids(body)
        except ValueError as e:
            return _err(400, str(e))
        return web.json_response({"model": body.get("model") or self.name, "token_ids": ids,
                                  "prompt_token_ids": ids, "count": len(ids),
                                  "max_model_len": self.cfg.sched.max_model_len})

    async def tokenize(self, req):
        body = await req.json()
        if "messages" in body:
            ids = self._chat_ids(body)
        else:
            ids = self.tok.encode(body.get("prompt", ""))
        return web.json_response({"tokens": ids, "count": len(ids), "max_model_len": self.cfg.sched.max_model_len})

    async def detokenize(self, req):
        body = await req.json()
        return web.json_response({"prompt": self.tok.decode(body.get("tokens", []))})

    # ------------------------------------------------------------ lifecycle
    async def pause(self, req):
        self.aeng.pause()
        return web.json_response({"paused": True})

    async def resume(self, req):
        self.aeng.resume()
        return web.json_response({"paused": False})

    # ------------------------------------------------------------ RL weight sync + sleep (M17)
    async def _ws(self, cmd: dict):
        try:
            res = await self.aeng.call(lambda e: e.weight_sync_cmd(cmd))
        except (RuntimeError, ValueError, KeyError, FileNotFoundError) as e:
            return _err(409 if isinstance(e, RuntimeError) else 400, str(e))
        return web.json_response(res)

    async def init_weight_update_group(self, req):
        b = await req.json()
        return await self._ws({"op": "init_group", "addr": b.get("master_address", "127.0.0.1"),
                               "port": int(b["master_port"]), "rank_offset": int(b.get("rank_offset", 1)),
                               "world_size": int(b["world_size"]), "backend": b.get("backend"),
                               "timeout_s": float(b.get("timeout_s", 300.0))})

    async def update_weights(self, req):
        b = await req.json()
        if "metas" in b:
            metas = [tuple(m) for m in b["metas"]]
        else:
            metas = list(zip(b["names"], b["dtypes"], b["shapes"]))
        cmd = {"op": "update_from_group", "metas": metas}
        if b.get("weights_version") is not None:  # the trainer's name for these weights (FS KV namespace)
            cmd["weights_version"] = str(b["weights_version"])
        r = await self._ws(cmd)
        self.aeng.wake.set()  # requests held after a level-2 wake-up can run now
        return r

    async def update_weights_from_disk(self, req):
        b = await req.json()
        cmd = {"op": "update_from_disk", "path": b["path"]}
        if b.get("weights_version") is not None:
            cmd["weights_version"] = str(b["weights_version"])
        r = await self._ws(cmd)
        self.aeng.wake.set()
        return r

    async def destroy_weight_update_group(self, req):
        return await self._ws({"op": "destroy_group"})

    async def sleep(self, req):
        level = int(req.query.get("level", 1))
        if req.can_read_body:
            level = int((await req.json()).get("level", level))
        return await self._ws({"op": "sleep", "level": level})

    async def wake_up(self, req):
        r = await self._ws({"op": "wake_up"})
        self.aeng.wake.set()
        return r

    async def is_sleeping(self, req):
        return web.json_response({"is_sleeping": bool(self.aeng.engine.sleeping),
                                  "level": self.aeng.engine.sleeping,
                                  "weights_pending": bool(self.aeng.engine.weights_pending)})

    # ------------------------------------------------------------ other OpenAI / vLLM / Anthropic surfaces
    async def _run_one(self, req, ids, params, prio=0, lora=0, mm=None):
        rid = req.headers.get("x-request-id") or f"req-{uuid.uuid4().hex}"
        toks, last = [], None
        async for o in self.aeng.generate(rid, ids, params, prio, None, lora, mm):
            toks.extend(o.new_token_ids)
            last = o
        return toks, last

    async def embeddings(self, req: web.Request):
        """OpenAI /v1/embeddings: last-token final hidden state, L2-normalised
        (the pooling of decoder-only embedding models)."""
        body = await req.json()
        inp = body.get("input")
        if inp is None:
            return _err(400, "input is required")
        try:
            if isinstance(inp, str) or (isinstance(inp, list) and inp and isinstance(inp[0], int)):
                inputs = [inp]
            else:
                inputs = list(inp)
            id_lists = [self.tok.encode(x) if isinstance(x, str) else list(x) for x in inputs]
        except (TypeError, ValueError) as e:
            return _err(400, str(e))
        params = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True, embed=True)
        res = await asyncio.gather(*[self._run_one(req, ids, params, lora=self._lora_id(body)) for ids in id_lists])
        data = [{"object": "embedding", "index": i, "embedding": (last.embedding if last else None) or []}
                for i, (_, last) in enumerate(res)]
        n = sum(len(x) for x in id_lists)
        return web.json_response({"object": "list", "data": data, "model": body.get("model") or self.name,
                                  "usage": {"prompt_tokens": n, "total_tokens": n}})

    async def responses(self, req: web.Request):
        """OpenAI Responses API (non-streaming): `input` (text or messages) +
        `instructions` -> one assistant message output item."""
        body = await req.json()
        inp = body.get("input")
        msgs = []
        if body.get("instructions"):
            msgs.append({"role": "system", "content": body["instructions"]})
        if isinstance(inp, str):
            msgs.append({"role": "user", "content": inp})
        elif isinstance(inp, list):
            for m in inp:
                c = m.get("content")
                if isinstance(c, list):
                    c = "".join(p.get("text", "") for p in c if isinstance(p, dict))
                msgs.append({"role": m.get("role", "user"), "content": c or ""})
        else:
            return _err(400, "input is required")
        ids = self.tok.encode(self.template.render(msgs, True))
        try:
            params = SamplingParams.from_openai(dict(body, max_tokens=body.get("max_output_tokens")),
                                                default_max=max(1, self.cfg.sched.max_model_len - len(ids) - 1),
                                                vocab_size=self._vocab)
        except (ValueError, TypeError) as e:
            return _err(400, str(e))
        toks, last = await self._run_one(req, ids, params, lora=self._lora_id(body))
        text = self.tok.decode(toks)
        rid = f"resp_{uuid.uuid4().hex}"
        return web.json_response({
            "id": rid, "object": "response", "created_at": int(time.time()),
            "status": "completed" if last and last.finish_reason != "error" else "failed",
            "model": body.get("model") or self.name,
            "output": [{"type": "message", "id": f"msg_{uuid.uuid4().hex}", "status": "completed",
                        "role": "assistant", "content": [{"type": "output_text", "text": text, "annotations": []}]}],
            "usage": {"input_tokens": len(ids), "output_tokens": len(toks), "total_tokens": len(ids) + len(toks)}})

    async def messages(self, req: web.Request):
        """Anthropic Messages API: system + messages with text (and base64 image)
        blocks -> one assistant text block; ``stream: true`` answers with the
        Anthropic SSE event sequence (message_start, content_block_start,
        content_block_delta x N, content_block_stop, message_delta, message_stop;
        reference docs/api-reference/epp-http-apis.md:238-300)."""
        body = await req.json()
        msgs = []
        sysm = body.get("system")
        if isinstance(sysm, list):
            sysm = "".join(b.get("text", "") for b in sysm if isinstance(b, dict))
        if sysm:
            msgs.append({"role": "system", "content": sysm})
        for m in body.get("messages") or []:
            c = m.get("content")
            if isinstance(c, list):
                parts = []
                for b in c:
                    if b.get("type") == "text":
                        parts.append({"type": "text", "text": b.get("text", "")})
                    elif b.get("type") == "image" and (b.get("source") or {}).get("type") == "base64":
                        src = b["source"]
                        parts.append({"type": "image_url", "image_url": {
                            "url": f"data:{src.get('media_type', 'image/png')};base64,{src.get('data', '')}"}})
                c = parts
            msgs.append({"role": m.get("role", "user"), "content": c})
        if not msgs:
            return _err(400, "messages is required")
        chat_body = {"messages": msgs, "max_tokens": body.get("max_tokens", 16),
                     "temperature": body.get("temperature", 1.0), "top_p": body.get("top_p", 1.0),
                     "top_k": body.get("top_k", 0), "stop": body.get("stop_sequences") or []}
        try:
            mm = None
            if self.mm is not None and self._has_images(chat_body):
                ids, mm = await self._chat_mm(chat_body, req.headers)
            else:
                ids = self._chat_ids(chat_body)
            params = SamplingParams.from_openai(chat_body, vocab_size=self._vocab)
        except (ValueError, TypeError) as e:
            return _err(400, str(e))
        if body.get("stream"):
            return await self._stream_messages(req, body, ids, params, mm)
        toks, last = await self._run_one(req, ids, params, lora=self._lora_id(body), mm=mm)
        text = self.tok.decode(toks)
        stop_seq = None
        for s in params.stop:
            k = text.find(s)
            if k >= 0:
                text, stop_seq = text[:k], s
        reason = "stop_sequence" if stop_seq else ("max_tokens" if last and last.finish_reason == "length"
                                                   else "end_turn")
        return web.json_response({"id": f"msg_{uuid.uuid4().hex}", "type": "message", "role": "assistant",
                                  "model": body.get("model") or self.name,
                                  "content": [{"type": "text", "text": text}], "stop_reason": reason,
                                  "stop_sequence": stop_seq,
                                  "usage": {"input_tokens": len(ids), "output_tokens": len(toks)}})

    async def _stream_messages(self, req, body, ids, params, mm):
        rid = req.headers.get("x-request-id") or f"req-{uuid.uuid4().hex}"
        mid = f"msg_{uuid.uuid4().hex}"
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream", "Cache-Control": "no-cache"})
        await resp.prepare(req)

        async def event(name, data):
            await resp.write(f"event: {name}\ndata: {json.dumps(data)}\n\n".encode())

        await event("message_start", {"type": "message_start", "message": {
            "id": mid, "type": "message", "role": "assistant", "model": body.get("model") or self.name,
            "content": [], "stop_reason": None, "stop_sequence": None,
            "usage": {"input_tokens": len(ids), "output_tokens": 0}}})
        await event("content_block_start", {"type": "content_block_start", "index": 0,
                                            "content_block": {"type": "text", "text": ""}})
        await event("ping", {"type": "ping"})
        toks: list[int] = []
        sent, stop_seq, last = "", None, None
        try:
            async for o in self.aeng.generate(rid, ids, params, 0, None, self._lora_id(body), mm):
                toks.extend(o.new_token_ids)
                last = o
                text = self.tok.decode(toks)
                for s in params.stop:
                    k = text.find(s)
                    if k >= 0:
                        text, stop_seq = text[:k], s
                delta = text[len(sent):] if text.startswith(sent) else ""
                sent = text
                if delta:
                    await event("content_block_delta", {"type": "content_block_delta", "index": 0,
                                                        "delta": {"type": "text_delta", "text": delta}})
                if stop_seq is not None:
                    self.aeng.abort(rid)
                    break
        except (ConnectionResetError, asyncio.CancelledError):
            self.aeng.abort(rid)
            raise
        except Exception as e:  # noqa: BLE001
            self.aeng.abort(rid)
            await event("error", {"type": "error", "error": {"type": "api_error", "message": str(e)}})
            await resp.write_eof()
            return resp
        reason = "stop_sequence" if stop_seq else ("max_tokens" if last and last.finish_reason == "length"
                                                   else "end_turn")
        await event("content_block_stop", {"type": "content_block_stop", "index": 0})
        await event("message_delta", {"type": "message_delta",
                                      "delta": {"stop_reason": reason, "stop_sequence": stop_seq},
                                      "usage": {"output_tokens": len(toks)}})
        await event("message_stop", {"type": "message_stop"})
        await resp.write_eof()
        return resp

    async def generate_tokens(self, req: web.Request):
        """vLLM token-in / token-out generate API (`/inference/v1/generate`, the
        router's vllmgrpc-style path): {"token_ids"|"prompt", "sampling_params"}."""
        body = await req.json()
        if "token_ids" in body:
            try:
                ids = self._token_ids(body["token_ids"])
            except (ValueError, TypeError) as e:
                return _err(400, str(e))
        elif isinstance(body.get("prompt"), str):
            ids = self.tok.encode(body["prompt"])
        else:
            return _err(400, "token_ids or prompt is required")
        sp = dict(body.get("sampling_params") or {})
        params = SamplingParams.from_openai(sp, default_max=16, vocab_size=self._vocab)
        toks, last = await self._run_one(req, ids, params, lora=self._lora_id(body))
        return web.json_response({"request_id": req.headers.get("x-request-id"), "prompt_token_ids": ids,
                                  "choices": [{"index": 0, "token_ids": toks,
                                               "finish_reason": last.finish_reason if last else "abort"}],
                                  "usage": {"prompt_tokens": len(ids), "completion_tokens": len(toks)}})

    # ------------------------------------------------------------ resilience (IRO)
    def faults(self) -> list[dict]:
        out = []
        if self.aeng.dead is not None:
            out.append({"kind": "engine_dead", "detail": repr(self.aeng.dead)})
        conn = self.aeng.engine.connector
        ag = getattr(conn, "agent", None)
        if ag is not None:
            for peer, st in ag.peer_status().items():
                if st == "dead":
                    out.append({"kind": "kv_peer_unreachable", "detail": peer})
        return out

    def _publish_fault(self, action: str, faults: list[dict]):
        pub = getattr(self, "kv_event_publisher", None)
        if pub is not None:
            pub.publish_batch({"ts": time.time(), "events": [{"type": "vllm_fault", "action": action,
                                                              "faults": faults}]},
                              topic=f"fault@{self.name}")

    async def _fault_monitor(self):
        """Engine-initiated fault notification (the ``vllm_fault`` PUB of
        inference-resilience-operator.md:176-186): publish when the fault set
        changes, so an operator reacts without polling ``/fault_tolerance/status``."""
        last: list[dict] = []
        period = float(os.environ.get("LLMD_FAULT_POLL_S", "1.0"))
        while True:
            await asyncio.sleep(period)
            cur = self.faults()
            if cur != last:
                self._publish_fault("detected" if cur else "cleared", cur)
                last = cur

    async def _start_fault_monitor(self, _app):
        self._fault_task = asyncio.get_running_loop().create_task(self._fault_monitor())

    async def _stop_fault_monitor(self, _app):
        t = getattr(self, "_fault_task", None)
        if t is not None:
            t.cancel()

    async def ft_status(self, req):
        faults = self.faults()
        eng = self.aeng.engine
        state = "faulted" if faults else ("paused" if eng.paused else "healthy")
        return web.json_response({"status": state, "faults": faults, "paused": eng.paused,
                                  "accepting": self.aeng.accepting, "num_running": eng.sched.num_running,
                                  "num_waiting": eng.sched.num_waiting})

    async def ft_apply(self, req):
        """Recovery actions: pause | resume | retry | drain {timeout} | abort_all |
        reset_prefix_cache. ``retry`` is the operator's answer to a transient,
        engine-internal fault: re-probe the KV-transfer peers, then resume."""
        body = await req.json()
        act = body.get("action")
        if act == "pause":
            self.aeng.pause()
        elif act == "retry":
            ag = getattr(self.aeng.engine.connector, "agent", None)
            if ag is not None:
                await asyncio.get_running_loop().run_in_executor(None, ag.heartbeat_once)
            self.aeng.accepting = True
            self.aeng.resume()
        elif act == "resume":
            self.aeng.accepting = True
            self.aeng.resume()
        elif act == "drain":
            await self.aeng.drain(float(body.get("timeout", 30)))
        elif act == "abort_all":
            for rid in list(self.aeng.streams):
                self.aeng.abort(rid)
        elif act == "reset_prefix_cache":
            await self.aeng.call(lambda e: e.reset_prefix_cache())
        else:
            return _err(400, f"unknown action {act!r}")
        self._publish_fault(act, self.faults())
        return web.json_response({"applied": act})

    async def is_paused(self, req):
        return web.json_response({"is_paused": self.aeng.engine.paused})

    async def reset_prefix_cache(self, req):
        await self.aeng.call(lambda e: e.reset_prefix_cache())
        return web.json_response({"status": "ok"})

    async def load_lora(self, req):
        if self.lora is None:
            return _err(400, "LoRA is not enabled (--enable-lora)")
        body = await req.json()
        try:
            await self.aeng.call(lambda e: self.lora.load(body["lora_name"], body.get("lora_path")))
        except Exception as e:  # noqa: BLE001
            return _err(400, str(e))
        return web.Response(text=f"Success: LoRA adapter '{body['lora_name']}' added successfully.")

    async def unload_lora(self, req):
        if self.lora is None:
            return _err(400, "LoRA is not enabled (--enable-lora)")
        body = await req.json()
        await self.aeng.call(lambda e: self.lora.unload(body["lora_name"]))
        return web.Response(text=f"Success: LoRA adapter '{body['lora_name']}' removed successfully.")


def build_server(cfg: EngineConfig, engine=None, opts: Optional[ServingOptions] = None):
    from llmd_amd.engine.engine import LLMEngine

    eng = engine or LLMEngine(cfg)
    aeng = AsyncEngine(eng)
    srv = OpenAIServer(aeng, cfg, lora_manager=eng.lora, opts=opts)
    if cfg.kv_events_config and cfg.kv_events_config.get("enable_kv_cache_events"):
        from .kv_events import KVEventPublisher

        pub = KVEventPublisher.from_config(cfg.kv_events_config, cfg.served_name, cfg.cache.block_size)
        eng.event_sink = pub.publish
        srv.kv_event_publisher = pub
    if eng.connector is not None:
        srv.extra_metrics.append(eng.connector.render_metrics)
    if eng.offload is not None:
        srv.extra_metrics.append(lambda: eng.offload.render_metrics(cfg.served_name))
    return srv


def add_serving_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    """Front-end flags with vLLM's names (chat template, parsers, streaming,
    multimodal roles, tracing), plus logging flags accepted for compatibility."""
    p.add_argument("--chat-template", default=None, help="Jinja chat template (file or inline)")
    p.add_argument("--enable-auto-tool-choice", action="store_true")
    p.add_argument("--tool-call-parser", default=None, help="hermes | llama3_json | mistral | pythonic | openai")
    p.add_argument("--reasoning-parser", default=None, help="deepseek_r1 | qwen3 | granite | openai_gptoss")
    p.add_argument("--stream-interval", type=int, default=1, help="stream every N generated tokens")
    p.add_argument("--limit-mm-per-prompt", type=_json_arg_safe, default=None, help='e.g. {"image": 4}')
    p.add_argument("--mm-encoder-only", action="store_true",
                   help="encode role: serve /v1/encode + /v1/ec only (E/PD encoder worker)")
    p.add_argument("--language-model-only", action="store_true",
                   help="never run the local vision tower: image embeddings come from encode workers")
    p.add_argument("--ec-transfer-config", type=_json_arg_safe, default=None,
                   help='{"ec_connector": ..., "ec_role": "ec_producer" | "ec_consumer"}')
    p.add_argument("--mm-processor-cache-gb", type=float, default=None, help="encoder-cache size (GiB)")
    p.add_argument("--otlp-traces-endpoint", default=None)
    p.add_argument("--collect-detailed-traces", default=None,
                   help="model / worker / all: also emit roctx ranges for the engine phases")
    p.add_argument("--api-server-count", type=int, default=1)
    p.add_argument("--numa-bind", action="store_true", help="pin this process to its GPU's NUMA node")
    for f in ("--disable-access-log-for-endpoints", "--uvicorn-access-log-exclude-prefixes"):
        p.add_argument(f, default=None, help=argparse.SUPPRESS)
    p.add_argument("--disable-uvicorn-access-log", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--grpc-port", type=int, default=0,
                   help="also serve the vLLM gRPC engine API (vllm.grpc.engine.VllmEngine) on this port (h2c)")
    return p


def _json_arg_safe(s):
    return json.loads(s) if s else None


def serving_options_from_args(a) -> ServingOptions:
    if a.tool_call_parser or a.reasoning_parser:
        ChatOutputParser(a.reasoning_parser, a.tool_call_parser)  # validate names at start-up
    if a.enable_auto_tool_choice and not a.tool_call_parser:
        raise SystemExit("--enable-auto-tool-choice requires --tool-call-parser")
    ec = a.ec_transfer_config or {}
    if ec and ec.get("ec_role") not in (None, "ec_producer", "ec_consumer", "ec_both"):
        raise SystemExit(f"--ec-transfer-config: unknown ec_role {ec.get('ec_role')!r}")
    return ServingOptions(chat_template=a.chat_template, enable_auto_tool_choice=a.enable_auto_tool_choice,
                          tool_call_parser=a.tool_call_parser, reasoning_parser=a.reasoning_parser,
                          stream_interval=max(1, a.stream_interval), limit_mm_per_prompt=a.limit_mm_per_prompt,
                          mm_encoder_only=a.mm_encoder_only)


def _numa_bind(device_index: int):
    """Pin the process to the CPUs of the GPU's NUMA node (sysfs; best effort)."""
    import glob

    try:
        import torch

        bus = torch.cuda.get_device_properties(device_index).pci_bus_id
        node = int(open(glob.glob(f"/sys/bus/pci/devices/*{bus:02x}:00.0/numa_node")[0]).read())
        if node < 0:
            return
        cpus = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
        sel = set()
        for part in cpus.split(","):
            lo, _, hi = part.partition("-")
            sel.update(range(int(lo), int(hi or lo) + 1))
        os.sched_setaffinity(0, sel)
        log.info("numa-bind: GPU %d -> node %d (%d CPUs)", device_index, node, len(sel))
    except Exception as e:  # noqa: BLE001
        log.warning("numa-bind skipped: %s", e)


def main(argv=None):
    p = argparse.ArgumentParser("llmd-amd serve")
    add_engine_args(p)
    add_serving_args(p)
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--shutdown-timeout", type=float, default=0.0)
    p.add_argument("--log-level", default="info")
    a = p.parse_args(argv)
    logging.basicConfig(level=a.log_level.upper(), format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    opts = serving_options_from_args(a)
    if a.otlp_traces_endpoint:
        from llmd_amd.utils import tracing

        tracing.configure_otlp(a.otlp_traces_endpoint)
    if a.collect_detailed_traces:
        os.environ.setdefault("LLMD_ROCTX", "1")
    if a.api_server_count != 1:
        log.warning("--api-server-count %d: one API server process per engine here (asyncio front end)",
                    a.api_server_count)
    for f in ("attention_backend", "moe_backend"):
        if getattr(a, f, None):
            log.info("--%s %s ignored: the attention / MoE kernels are this repo's HIP kernels",
                     f.replace("_", "-"), getattr(a, f))
    cfg = engine_config_from_args(a)
    port = a.port
    pc = cfg.parallel
    if pc.tensor_parallel_size > 1 or pc.data_parallel_size > 1:
        # one process per GPU under torchrun (WORLD_SIZE = tp x dp); TP rank 0 of
        # each DP group serves, the others follow
        from llmd_amd.parallel.state import init_distributed

        st = init_distributed(tp_size=pc.tensor_parallel_size, backend=None if cfg.device == "cuda" else "gloo")
        if st.dp_size != pc.data_parallel_size:
            raise SystemExit(f"WORLD_SIZE {st.world_size} != --tensor-parallel-size {pc.tensor_parallel_size} x "
                             f"--data-parallel-size {pc.data_parallel_size}")
        local_dp = int(os.environ.get("LOCAL_WORLD_SIZE", st.world_size)) // pc.tensor_parallel_size
        if a.data_parallel_size_local is not None and a.data_parallel_size_local != local_dp:
            raise SystemExit(f"--data-parallel-size-local {a.data_parallel_size_local} != {local_dp} local DP "
                             "ranks under torchrun")
        if pc.data_parallel_size > 1:
            port = dp_rank_port(cfg, a.port, st.dp_rank)
        if st.tp_rank != 0:
            from llmd_amd.engine.tp_worker import run_follower

            run_follower(cfg, capture_graphs=not cfg.enforce_eager)
            return
    if a.numa_bind and cfg.device == "cuda":
        import torch

        _numa_bind(torch.cuda.current_device() if torch.cuda.is_initialized() else 0)
    srv = build_server(cfg, opts=opts)
    if srv.mm is not None:
        if a.language_model_only:
            srv.mm.has_tower = False
        if a.mm_processor_cache_gb:
            srv.mm.cache.max_bytes = int(a.mm_processor_cache_gb * (1 << 30))
    app = srv.app()

    async def on_shutdown(_app):
        if srv.mm is not None:
            await srv.mm.close()
        if a.shutdown_timeout > 0:
            await srv.aeng.drain(a.shutdown_timeout)
        srv.aeng.shutdown()

    app.on_shutdown.append(on_shutdown)
    if a.grpc_port:
        from . import vllm_grpc

        grpc_box = {}

        async def grpc_start(_app):
            grpc_box["s"], _ = await vllm_grpc.start_server(srv, a.grpc_port, a.host)

        async def grpc_stop(_app):
            if "s" in grpc_box:
                await grpc_box["s"].stop(grace=1.0)
        app.on_startup.append(grpc_start)
        app.on_shutdown.insert(0, grpc_stop)
    # keep-alive must exceed the sidecar's 90 s idle timeout (VLLM_HTTP_TIMEOUT_KEEP_ALIVE=120)
    keepalive = float(os.environ.get("VLLM_HTTP_TIMEOUT_KEEP_ALIVE", "120"))
    web.run_app(app, host=a.host, port=port, keepalive_timeout=keepalive, access_log=None,
                shutdown_timeout=max(a.shutdown_timeout, 1.0))


def dp_rank_port(cfg: EngineConfig, base_port: int, dp_rank: int) -> int:
    """Data parallelism with an external load balancer (the reference's
    multi-port DP-aware wide-EP: every DP rank is its own router endpoint,
    guides/wide-ep-lws/experimental-dp-aware/README.md:1-29, router targetPorts
    8000-8007): DP rank r serves the OpenAI API on ``base_port + r`` and
    publishes KV events on its own port (endpoint port + r). Wide-EP ranks
    (MoE + --enable-expert-parallel) step in lockstep (engine/engine.py)."""
    cfg.parallel.data_parallel_rank = dp_rank
    kc = cfg.kv_events_config
    if kc and kc.get("endpoint"):
        head, _, tail = kc["endpoint"].rpartition(":")
        if tail.isdigit():
            cfg.kv_events_config = dict(kc, endpoint=f"{head}:{int(tail) + dp_rank}")
    return base_port + dp_rank


if __name__ == "__main__":
    main()
