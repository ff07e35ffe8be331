"""Multimodal serving + encoder disaggregation (E/PD, E/P/D; SURVEY C27,
reference guides/multimodal-serving/e-disaggregation/README.md:1-46,252-321).

Roles
* **encode** worker (a multimodal server deployed with the
  ``llm-d.ai/role: encode`` label, picked by the router's ``encode-filter``):
  ``POST /v1/encode`` {"images": [url, ...]} encodes each image (or finds it in
  its encoder cache) and answers ``[{mm_hash, num_tokens, hidden}]``;
  ``GET /v1/ec/{mm_hash}`` streams the bf16 embedding bytes. That pair is the
  EC connector's XferReq/XferAck + data plane (the reference uses ZMQ control
  + NIXL data; one node needs no NIC path, HTTP keeps the CPU CI path).
* **prefill/decode** engine (same binary, role prefill/decode): a chat
  request with ``image_url`` parts is rendered with a run of
  ``image_token_id`` placeholders per image (count = the vision tower's
  (W/28)*(H/28)). Embeddings come from, in order: the local EC cache (by
  image hash), the encoders named in ``x-encoder-hosts-ports`` (set by the
  router's disagg profile handler / sidecar), or the local vision tower when
  the model has one (aggregated E+PD).

Prefix caching keys fold the image hashes in (Request.cache_extra), matching
the reference's mm ``extra_keys`` in KV events.
"""
from __future__ import annotations

import asyncio
import io
import logging
from collections import OrderedDict
from typing import Optional

import aiohttp
import numpy as np
import torch
from aiohttp import web

from llmd_amd.models.vision import MMInput, VisionConfig, load_image_bytes, mm_hash, num_image_tokens

log = logging.getLogger("llmd.mm")

ENCODER_HEADER = "x-encoder-hosts-ports"
IMG_MARK = "\x00<image>\x00"


class ECCache:
    """LRU of image hash -> embeddings (host bf16) bounded by bytes."""

    def __init__(self, max_bytes: int = 2 << 30):
        self.max_bytes = max_bytes
        self.bytes = 0
        self.d: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        self.hits = 0
        self.misses = 0

    def get(self, h: str) -> Optional[torch.Tensor]:
        t = self.d.get(h)
        if t is None:
            self.misses += 1
            return None
        self.d.move_to_end(h)
        self.hits += 1
        return t

    def put(self, h: str, t: torch.Tensor):
        if h in self.d:
            return
        t = t.detach().to("cpu", torch.bfloat16).contiguous()
        self.d[h] = t
        self.bytes += t.numel() * 2
        while self.bytes > self.max_bytes and len(self.d) > 1:
            _, old = self.d.popitem(last=False)
            self.bytes -= old.numel() * 2


def image_parts(messages: list[dict]) -> list[str]:
    urls = []
    for m in messages:
        c = m.get("content")
        if isinstance(c, list):
            for p in c:
                if isinstance(p, dict) and p.get("type") in ("image_url", "input_image"):
                    iu = p.get("image_url")
                    urls.append(iu.get("url") if isinstance(iu, dict) else (iu or p.get("url")))
    return urls


def mark_images(messages: list[dict]) -> list[dict]:
    """Copy of messages with each image part replaced by a text marker."""
    out = []
    for m in messages:
        c = m.get("content")
        if isinstance(c, list):
            parts = []
            for p in c:
                if isinstance(p, dict) and p.get("type") in ("image_url", "input_image"):
                    parts.append({"type": "text", "text": IMG_MARK})
                else:
                    parts.append(p)
            m = dict(m, content=parts)
        out.append(m)
    return out


def image_dims(b: bytes) -> tuple[int, int]:
    from PIL import Image

    with Image.open(io.BytesIO(b)) as im:
        return im.width, im.height


def build_prompt(text: str, tok, images: list[bytes], vcfg: VisionConfig, image_token_id: int):
    """Rendered chat text with IMG_MARK markers -> token ids with placeholder
    runs and the MMInput (no embeddings yet) of every image."""
    pieces = text.split(IMG_MARK)
    if len(pieces) - 1 != len(images):
        raise ValueError("image markers do not match image parts")
    ids: list[int] = []
    mm: list[MMInput] = []
    for i, piece in enumerate(pieces):
        if piece:
            ids.extend(tok.encode(piece))
        if i < len(images):
            n = num_image_tokens(*image_dims(images[i]), vcfg)
            mm.append(MMInput(offset=len(ids), length=n, mm_hash=mm_hash(images[i]), meta={"bytes": images[i]}))
            ids.extend([image_token_id] * n)
    return ids, mm


async def fetch_from_encoder(session: aiohttp.ClientSession, host_port: str, urls: list[str]) -> list[tuple]:
    """XferReq to an encode worker, then pull each embedding (data plane)."""
    base = f"http://{host_port}"
    async with session.post(base + "/v1/encode", json={"images": urls}) as r:
        if r.status != 200:
            raise RuntimeError(f"encoder {host_port} returned {r.status}: {await r.text()}")
        infos = (await r.json())["data"]
    out = []
    for info in infos:
        async with session.get(f"{base}/v1/ec/{info['mm_hash']}") as r:
            if r.status != 200:
                raise RuntimeError(f"encoder {host_port}: embedding {info['mm_hash'][:12]} missing")
            raw = await r.read()
        t = torch.from_numpy(np.frombuffer(raw, dtype=np.int16).copy()).view(torch.bfloat16)
        out.append((info["mm_hash"], t.view(info["num_tokens"], info["hidden"])))
    return out


class MultimodalFrontend:
    """Resolves image embeddings for a chat request (local cache, remote
    encoders, or the engine's own vision tower) and serves the encode role."""

    def __init__(self, aeng, cfg, tok):
        self.aeng = aeng
        self.cfg = cfg
        self.tok = tok
        mc = cfg.model_config
        self.vcfg = VisionConfig(**(mc.vision_config or {}))
        self.image_token_id = mc.image_token_id
        self.has_tower = mc.model_type == "llava"
        self.cache = ECCache()
        self._session: Optional[aiohttp.ClientSession] = None
        self.n_remote = 0
        self.n_local = 0

    @property
    def enabled(self) -> bool:
        return self.cfg.model_config.vision_config is not None

    async def session(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=120))
        return self._session

    async def close(self):
        if self._session is not None and not self._session.closed:
            await self._session.close()

    async def encode_local(self, b: bytes) -> torch.Tensor:
        if not self.has_tower:
            raise ValueError("this model has no vision tower and no encoder was given")
        t = await self.aeng.call(lambda eng: eng.runner.model.encode_image(b).cpu())
        self.n_local += 1
        return t

    async def prepare(self, body: dict, text: str, headers) -> tuple[list[int], list[MMInput]]:
        urls = image_parts(body.get("messages") or [])
        images = [load_image_bytes(u) for u in urls]
        ids, mm = build_prompt(text, self.tok, images, self.vcfg, self.image_token_id)
        missing = [i for i, it in enumerate(mm) if self.cache.get(it.mm_hash) is None]
        enc = [h.strip() for h in (headers.get(ENCODER_HEADER) or "").split(",") if h.strip()]
        if missing and enc:
            sess = await self.session()
            groups: dict[str, list[int]] = {}
            for j, i in enumerate(missing):  # spread images over the listed encoders
                groups.setdefault(enc[j % len(enc)], []).append(i)
            res = await asyncio.gather(*[fetch_from_encoder(sess, hp, [urls[i] for i in idx])
                                         for hp, idx in groups.items()])
            for got in res:
                for h, t in got:
                    self.cache.put(h, t)
                    self.n_remote += 1
        for it in mm:
            t = self.cache.get(it.mm_hash)
            if t is None:
                t = await self.encode_local(it.meta["bytes"])
                self.cache.put(it.mm_hash, t)
            if t.shape[0] != it.length:
                raise ValueError(f"image {it.mm_hash[:12]}: encoder produced {t.shape[0]} tokens, "
                                 f"prompt reserved {it.length}")
            it.embeds = t
            it.meta.pop("bytes", None)
        return ids, mm

    # ------------------------------------------------------------ encode role endpoints
    async def http_encode(self, req: web.Request):
        try:
            body = await req.json()
            urls = list(body.get("images") or [])
            out = []
            for u in urls:
                b = load_image_bytes(u)
                h = mm_hash(b)
                t = self.cache.get(h)
                if t is None:
                    t = await self.encode_local(b)
                    self.cache.put(h, t)
                out.append({"mm_hash": h, "num_tokens": int(t.shape[0]), "hidden": int(t.shape[1]),
                            "dtype": "bfloat16"})
        except ValueError as e:
            return web.json_response({"error": {"message": str(e), "code": 400}}, status=400)
        return web.json_response({"object": "list", "data": out})

    async def http_ec(self, req: web.Request):
        t = self.cache.get(req.match_info["mm_hash"])
        if t is None:
            return web.json_response({"error": {"message": "unknown mm_hash", "code": 404}}, status=404)
        return web.Response(body=t.view(torch.int16).numpy().tobytes(), content_type="application/octet-stream")

    def metrics_text(self) -> str:
        name = self.cfg.served_name
        return (f'llmd:ec_cache_hits_total{{model_name="{name}"}} {self.cache.hits}\n'
                f'llmd:ec_cache_misses_total{{model_name="{name}"}} {self.cache.misses}\n'
                f'llmd:ec_remote_fetches_total{{model_name="{name}"}} {self.n_remote}\n'
                f'llmd:ec_local_encodes_total{{model_name="{name}"}} {self.n_local}\n')
