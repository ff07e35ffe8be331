"""Request parsers (docs/architecture/core/router/epp/request-handling.md:71-75,
docs/api-reference/epp-http-apis.md)."""
from __future__ import annotations

import json

from .. import headers as H
from ..types import CIHeaders, InferenceRequest
from ..multimodal import TokenEstimator, asset_hash, image_url_of, virtual_segment
from .base import Parser, register

_DEFAULT_EST = TokenEstimator()

OPENAI_PATHS = ("/v1/completions", "/v1/chat/completions", "/v1/embeddings", "/v1/responses",
                "/v1/conversations", "/v1/messages", "/inference/v1/generate")


def _content_text(c, est: TokenEstimator, assets: list) -> str:
    if not isinstance(c, list):
        return c or ""
    out = []
    for p in c:
        if not isinstance(p, dict):
            continue
        url = image_url_of(p)
        if url:  # multimodal asset -> virtual segment of its estimated token footprint
            assets.append((asset_hash(url), est.tokens(url)))
            out.append(virtual_segment(url, est))
        else:
            out.append(p.get("text", ""))
    return "".join(out)


def _flatten_prompt(body: dict, est: TokenEstimator = _DEFAULT_EST, assets: list | None = None) -> str:
    assets = [] if assets is None else assets
    if "messages" in body:
        parts = []
        for m in body.get("messages") or []:
            parts.append(f"<{m.get('role', '')}>{_content_text(m.get('content'), est, assets)}")
        return "".join(parts)
    if "input" in body:  # responses / embeddings
        i = body["input"]
        return i if isinstance(i, str) else json.dumps(i)
    p = body.get("prompt", "")
    if isinstance(p, list):
        if p and isinstance(p[0], int):
            return " ".join(map(str, p))
        return "".join(x if isinstance(x, str) else " ".join(map(str, x)) for x in p)
    if p is not None and not isinstance(p, str):  # a malformed request is the client's error (400)
        raise ValueError(f"prompt must be a string or a list, got {type(p).__name__}")
    return p or ""


@register("openai-parser")
class OpenAIParser(Parser):
    def parse(self, path, body: bytes, headers) -> InferenceRequest:
        try:
            d = json.loads(body) if body else {}
        except json.JSONDecodeError as e:
            raise ValueError(f"invalid JSON body: {e}") from e
        if not isinstance(d, dict):
            raise ValueError("JSON object expected")
        h = headers if isinstance(headers, CIHeaders) else CIHeaders(dict(headers))
        req = InferenceRequest(path=path, body=d, headers=h, raw_size=len(body))
        req.model = d.get("model", "") or ""
        req.target_model = req.model
        est = getattr(self, "_est", None)
        if est is None:
            est = self._est = TokenEstimator.from_params((getattr(self, "params", None) or {}).get("multimodal"))
        assets: list = []
        req.prompt = _flatten_prompt(d, est, assets)
        req.mm_assets = assets
        p = d.get("prompt")
        if isinstance(p, list) and p and isinstance(p[0], int):
            req.token_ids = list(p)
        req.stream = bool(d.get("stream", False))
        return req


@register("passthrough-parser")
class PassthroughParser(Parser):
    def parse(self, path, body, headers):
        h = headers if isinstance(headers, CIHeaders) else CIHeaders(dict(headers))
        try:
            d = json.loads(body) if body else {}
        except json.JSONDecodeError:
            d = {}
        req = InferenceRequest(path=path, body=d if isinstance(d, dict) else {}, headers=h, raw_size=len(body))
        req.model = req.body.get("model", "") if isinstance(req.body, dict) else ""
        req.target_model = req.model
        return req


@register("vllmgrpc-parser")
class VllmGrpcParser(OpenAIParser):
    """vLLM gRPC ``VllmEngine/Generate`` and ``/Embed``
    (docs/api-reference/epp-grpc-apis.md:9-14): the body is the gRPC-framed
    protobuf message (5-byte length prefix) of an h2c request, as the ext_proc
    stream (Envoy) or the router's gRPC data plane (router/grpc_proxy.py) hands
    it over. ``tokenized.input_ids`` become the request's exact tokens for
    prefix scoring (``text`` input: the text); the body is forwarded unchanged
    (no model rewrite: the message has no model field). Other paths: the
    OpenAI parser, plus JSON ``token_ids`` (/inference/v1/generate)."""

    def parse(self, path, body, headers):
        from llmd_amd.serving import vllm_grpc as vg

        if path not in vg.PATHS:
            req = super().parse(path, body, headers)
            if "token_ids" in req.body:
                req.token_ids = list(req.body["token_ids"])
            return req
        msgs = vg.unframe(bytes(body))
        if len(msgs) != 1:
            raise ValueError(f"expected one gRPC message, got {len(msgs)}")
        h = headers if isinstance(headers, CIHeaders) else CIHeaders(dict(headers))
        from google.protobuf.message import DecodeError

        try:
            if path == vg.GENERATE:
                m = vg.PB["GenerateRequest"].FromString(msgs[0])
            else:
                m = vg.PB["EmbedRequest"].FromString(msgs[0])
        except DecodeError as e:
            raise ValueError(f"invalid {path} message: {e}") from e
        req = InferenceRequest(path=path, body={"grpc_method": path.rsplit("/", 1)[1]}, headers=h,
                               raw_size=len(body))
        req.data["grpc"] = True
        req.model = h.get("x-llm-d-model", "") or ""
        req.target_model = req.model
        if path == vg.GENERATE and m.WhichOneof("input") == "text":
            req.prompt = m.text
        else:
            req.token_ids = list(m.tokenized.input_ids)
            req.prompt = m.tokenized.original_text or " ".join(map(str, req.token_ids))
        req.stream = bool(getattr(m, "stream", False))
        if m.request_id:
            req.request_id = m.request_id
        return req
