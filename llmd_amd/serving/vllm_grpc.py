"""vLLM gRPC engine API (``vllm.grpc.engine.VllmEngine``: Generate / Embed /
HealthCheck), served by the engine next to its OpenAI HTTP API, and the
wire helpers the router's ``vllmgrpc-parser`` and gRPC data plane use
(reference docs/api-reference/epp-gRPC-apis.md:9-57).

* Generate: token-out. Input is ``tokenized.input_ids`` (or ``text``, which the
  engine tokenizes); ``stream: false`` answers one ``complete`` message
  (``output_ids``, ``finish_reason``, prompt / completion token counts),
  ``stream: true`` a ``chunk`` per engine step (``token_ids``) and a final
  ``complete``.
* Embed: pre-tokenized input -> ``embedding`` (last-token final hidden state,
  L2-normalised, as /v1/embeddings), ``prompt_tokens``, ``embedding_dim``.

No protoc in this image: the descriptors are built in code. Field numbers
follow the llm-d-router ``vllm_engine.proto`` layout as far as the public docs
pin it (the reference repo does not ship the .proto: parity of the numbers is
unpinned; the server, parser and client here share this one definition).
"""
from __future__ import annotations

import asyncio
import logging
import struct
import time
import uuid
from typing import Optional

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

log = logging.getLogger("llmd.vllm_grpc")

SERVICE = "vllm.grpc.engine.VllmEngine"
GENERATE = f"/{SERVICE}/Generate"
EMBED = f"/{SERVICE}/Embed"
HEALTH = f"/{SERVICE}/HealthCheck"
PATHS = (GENERATE, EMBED)

_F = descriptor_pb2.FieldDescriptorProto
_T = {"string": _F.TYPE_STRING, "bool": _F.TYPE_BOOL, "int32": _F.TYPE_INT32, "uint32": _F.TYPE_UINT32,
      "float": _F.TYPE_FLOAT, "msg": _F.TYPE_MESSAGE}


def _msg(fdp, name, fields, oneofs=()):
    m = fdp.message_type.add(name=name)
    for o in oneofs:
        m.oneof_decl.add(name=o)
    for f in fields:
        fname, num, typ = f[:3]
        tname = f[3] if len(f) > 3 else None
        rep = f[4] if len(f) > 4 else False
        oneof = f[5] if len(f) > 5 else None
        fd = m.field.add(name=fname, number=num, type=_T[typ],
                         label=_F.LABEL_REPEATED if rep else _F.LABEL_OPTIONAL)
        if tname:
            fd.type_name = tname
        if oneof is not None:
            fd.oneof_index = oneofs.index(oneof)
    return m


def _build():
    pool = descriptor_pool.DescriptorPool()
    fd = descriptor_pb2.FileDescriptorProto(name="vllm_engine.proto", package="vllm.grpc.engine", syntax="proto3")
    P = ".vllm.grpc.engine."
    _msg(fd, "TokenizedInput", [("original_text", 1, "string"), ("input_ids", 2, "uint32", None, True)])
    _msg(fd, "SamplingParams", [
        ("temperature", 1, "float"), ("top_p", 2, "float"), ("top_k", 3, "uint32"), ("min_p", 4, "float"),
        ("frequency_penalty", 5, "float"), ("presence_penalty", 6, "float"), ("repetition_penalty", 7, "float"),
        ("max_tokens", 8, "uint32"), ("min_tokens", 9, "uint32"), ("stop", 10, "string", None, True),
        ("stop_token_ids", 11, "uint32", None, True), ("skip_special_tokens", 12, "bool"),
        ("ignore_eos", 14, "bool"), ("n", 15, "uint32"), ("seed", 16, "int32")])
    _msg(fd, "GenerateRequest", [
        ("request_id", 1, "string"),
        ("tokenized", 2, "msg", P + "TokenizedInput", False, "input"),
        ("text", 3, "string", None, False, "input"),
        ("sampling_params", 4, "msg", P + "SamplingParams"), ("stream", 5, "bool")], oneofs=("input",))
    _msg(fd, "GenerateStreamChunk", [("token_ids", 1, "uint32", None, True), ("prompt_tokens", 2, "uint32"),
                                     ("completion_tokens", 3, "uint32"), ("cached_tokens", 4, "uint32")])
    _msg(fd, "GenerateComplete", [("output_ids", 1, "uint32", None, True), ("finish_reason", 2, "string"),
                                  ("prompt_tokens", 3, "uint32"), ("completion_tokens", 4, "uint32"),
                                  ("cached_tokens", 5, "uint32")])
    _msg(fd, "GenerateError", [("message", 1, "string"), ("http_status_code", 2, "string"),
                               ("details", 3, "string")])
    _msg(fd, "GenerateResponse", [
        ("chunk", 1, "msg", P + "GenerateStreamChunk", False, "response"),
        ("complete", 2, "msg", P + "GenerateComplete", False, "response"),
        ("error", 3, "msg", P + "GenerateError", False, "response")], oneofs=("response",))
    _msg(fd, "EmbedRequest", [("request_id", 1, "string"), ("tokenized", 2, "msg", P + "TokenizedInput")])
    _msg(fd, "EmbedResponse", [("embedding", 1, "float", None, True), ("prompt_tokens", 2, "uint32"),
                               ("embedding_dim", 3, "uint32")])
    _msg(fd, "HealthCheckRequest", [])
    _msg(fd, "HealthCheckResponse", [("healthy", 1, "bool"), ("message", 2, "string")])
    pool.Add(fd)
    names = ["TokenizedInput", "SamplingParams", "GenerateRequest", "GenerateStreamChunk", "GenerateComplete",
             "GenerateError", "GenerateResponse", "EmbedRequest", "EmbedResponse", "HealthCheckRequest",
             "HealthCheckResponse"]
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName("vllm.grpc.engine." + n)) for n in names}


PB = _build()


# ------------------------------------------------------------------ gRPC wire framing
def frame(msg_bytes: bytes) -> bytes:
    """One length-prefixed gRPC message (uncompressed)."""
    return b"\x00" + struct.pack(">I", len(msg_bytes)) + msg_bytes


def unframe(buf: bytes) -> list[bytes]:
    """Split a gRPC body (HTTP/2 DATA payload) into its messages; a trailing
    partial frame is ignored (more DATA to come)."""
    out, i = [], 0
    while i + 5 <= len(buf):
        if buf[i] != 0:
            raise ValueError("compressed gRPC messages are not supported")
        n = struct.unpack(">I", buf[i + 1:i + 5])[0]
        if i + 5 + n > len(buf):
            break
        out.append(buf[i + 5:i + 5 + n])
        i += 5 + n
    return out


def usage_of_responses(msgs: list[bytes]) -> dict:
    """Usage of a Generate response stream (the router's response accounting):
    completion tokens counted from the chunks, or taken from ``complete``."""
    u = {"prompt_tokens": 0, "completion_tokens": 0}
    n_chunk = 0
    for m in msgs:
        r = PB["GenerateResponse"].FromString(m)
        kind = r.WhichOneof("response")
        if kind == "chunk":
            n_chunk += len(r.chunk.token_ids)
            u["prompt_tokens"] = r.chunk.prompt_tokens or u["prompt_tokens"]
        elif kind == "complete":
            u["prompt_tokens"] = r.complete.prompt_tokens or u["prompt_tokens"]
            u["completion_tokens"] = r.complete.completion_tokens or len(r.complete.output_ids) or n_chunk
    if not u["completion_tokens"]:
        u["completion_tokens"] = n_chunk
    u["total_tokens"] = u["prompt_tokens"] + u["completion_tokens"]
    return u


def sampling_from_proto(sp, vocab_size: Optional[int] = None):
    from llmd_amd.engine.request import SamplingParams

    body = {"max_tokens": sp.max_tokens if sp.max_tokens else 16,
            "temperature": sp.temperature,  # proto3 scalar: unset = 0 = greedy (token-out API)
            "top_p": sp.top_p if sp.top_p > 0 else 1.0, "top_k": sp.top_k, "min_p": sp.min_p,
            "frequency_penalty": sp.frequency_penalty, "presence_penalty": sp.presence_penalty,
            "repetition_penalty": sp.repetition_penalty if sp.repetition_penalty > 0 else 1.0,
            "min_tokens": sp.min_tokens, "stop": list(sp.stop), "stop_token_ids": list(sp.stop_token_ids),
            "ignore_eos": sp.ignore_eos, "seed": sp.seed if sp.seed else None}
    return SamplingParams.from_openai(body, vocab_size=vocab_size)


# ------------------------------------------------------------------ engine-side service
class VllmEngineService:
    """grpc.aio handlers over the API server's AsyncEngine + tokenizer."""

    def __init__(self, api):
        self.api = api  # serving.api_server.APIServer (aeng, tok, cfg)

    def _ids(self, req) -> list[int]:
        if req.WhichOneof("input") == "tokenized":
            return self.api._token_ids(list(req.tokenized.input_ids))
        if req.WhichOneof("input") == "text":
            return self.api.tok.encode(req.text)
        raise ValueError("GenerateRequest needs tokenized.input_ids or text")

    async def generate(self, req, context):
        GR = PB["GenerateResponse"]
        try:
            ids = self._ids(req)
            sp = req.sampling_params
            params = sampling_from_proto(sp, self.api._vocab)
        except (ValueError, TypeError) as e:
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            return
        if not ids or len(ids) + 1 > self.api.cfg.sched.max_model_len:
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, "prompt empty or longer than max_model_len")
            return
        md = dict(context.invocation_metadata() or ())
        rid = req.request_id or md.get("x-request-id") or f"grpc-{uuid.uuid4().hex}"
        prio = 0
        out: list[int] = []
        last = None
        try:
            async for o in self.api.aeng.generate(rid, ids, params, prio, None, 0, None):
                out.extend(o.new_token_ids)
                last = o
                if req.stream and o.new_token_ids:
                    yield GR(chunk=PB["GenerateStreamChunk"](token_ids=o.new_token_ids, prompt_tokens=len(ids),
                                                             completion_tokens=len(o.new_token_ids),
                                                             cached_tokens=o.num_cached_tokens))
        except asyncio.CancelledError:
            self.api.aeng.abort(rid)
            raise
        c = PB["GenerateComplete"](finish_reason=(last.finish_reason if last else None) or "abort",
                                   prompt_tokens=len(ids), completion_tokens=len(out),
                                   cached_tokens=last.num_cached_tokens if last else 0)
        if not req.stream:
            c.output_ids.extend(out)
        yield GR(complete=c)

    async def embed(self, req, context):
        from llmd_amd.engine.request import SamplingParams

        try:
            ids = self.api._token_ids(list(req.tokenized.input_ids))
        except (ValueError, TypeError) as e:
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            return None
        if not ids:
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, "Embed needs tokenized.input_ids")
            return None
        rid = req.request_id or f"grpc-emb-{uuid.uuid4().hex}"
        last = None
        async for o in self.api.aeng.generate(rid, ids, SamplingParams(max_tokens=1, temperature=0.0,
                                                                       ignore_eos=True, embed=True),
                                              0, None, 0, None):
            last = o
        emb = list((last.embedding if last else None) or [])
        return PB["EmbedResponse"](embedding=emb, prompt_tokens=len(ids), embedding_dim=len(emb))

    async def health(self, req, context):
        dead = getattr(self.api.aeng, "dead", False)
        return PB["HealthCheckResponse"](healthy=not dead, message="dead" if dead else "ok")

    def handler(self):
        return grpc.method_handlers_generic_handler(SERVICE, {
            "Generate": grpc.unary_stream_rpc_method_handler(
                self.generate, request_deserializer=PB["GenerateRequest"].FromString,
                response_serializer=PB["GenerateResponse"].SerializeToString),
            "Embed": grpc.unary_unary_rpc_method_handler(
                self.embed, request_deserializer=PB["EmbedRequest"].FromString,
                response_serializer=PB["EmbedResponse"].SerializeToString),
            "HealthCheck": grpc.unary_unary_rpc_method_handler(
                self.health, request_deserializer=PB["HealthCheckRequest"].FromString,
                response_serializer=PB["HealthCheckResponse"].SerializeToString)})


async def start_server(api, port: int, host: str = "0.0.0.0"):
    """Start the VllmEngine gRPC server on the running event loop; returns (server, bound port)."""
    s = grpc.aio.server(options=[("grpc.max_receive_message_length", 64 << 20),
                                 ("grpc.max_send_message_length", 64 << 20)])
    s.add_generic_rpc_handlers((VllmEngineService(api).handler(),))
    bound = s.add_insecure_port(f"{host}:{port}")
    await s.start()
    log.info("vLLM gRPC engine API on :%d", bound)
    return s, bound


# ------------------------------------------------------------------ client helpers (tests, tools)
class Client:
    def __init__(self, target: str):
        self.ch = grpc.aio.insecure_channel(target)
        self._gen = self.ch.unary_stream(GENERATE, request_serializer=PB["GenerateRequest"].SerializeToString,
                                         response_deserializer=PB["GenerateResponse"].FromString)
        self._emb = self.ch.unary_unary(EMBED, request_serializer=PB["EmbedRequest"].SerializeToString,
                                        response_deserializer=PB["EmbedResponse"].FromString)

    async def generate(self, input_ids=None, text=None, max_tokens=16, temperature=0.0, stream=False,
                       metadata=(), **sp):
        req = PB["GenerateRequest"](request_id=f"c-{uuid.uuid4().hex[:8]}", stream=stream,
                                    sampling_params=PB["SamplingParams"](max_tokens=max_tokens,
                                                                         temperature=temperature, **sp))
        if input_ids is not None:
            req.tokenized.input_ids.extend(input_ids)
        else:
            req.text = text or ""
        t0 = time.monotonic()
        return [r async for r in self._gen(req, metadata=tuple(metadata))], time.monotonic() - t0

    async def embed(self, input_ids, metadata=()):
        return await self._emb(PB["EmbedRequest"](request_id="e", tokenized=PB["TokenizedInput"](
            input_ids=input_ids)), metadata=tuple(metadata))

    async def close(self):
        await self.ch.close()
