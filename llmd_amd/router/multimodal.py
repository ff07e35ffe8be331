"""Multimodal-aware prefix scoring (reference
docs/well-lit-paths/workloads/multimodal-serving.md:46-70).

The approximate prefix index works on characters, so every image in a chat
request is replaced by a deterministic virtual segment whose identity is the
asset hash and whose length is its estimated token footprint:

* dimension strategy (Qwen-VL): tokens = ceil(W * H / factor), factor 784
  (28x28, Qwen2.5-VL) or 1024 (32x32, Qwen3.5-VL); W/H are read from the
  image header of data: URLs (PNG, JPEG, GIF, WebP); remote URLs fall back
  to the fixed allocation;
* fixed strategy (Gemma 4): a configured count (70/140/280/560/1120).

Two requests carrying the same image then share prefix blocks of the right
size, and a different image breaks the match at the right position.
"""
from __future__ import annotations

import base64
import hashlib
import math
import struct
from dataclasses import dataclass
from typing import Optional

CHARS_PER_TOKEN = 4


def _dims_png(b: bytes):
    if b[:8] == b"\x89PNG\r\n\x1a\n" and b[12:16] == b"IHDR":
        return struct.unpack(">II", b[16:24])
    return None


def _dims_gif(b: bytes):
    if b[:6] in (b"GIF87a", b"GIF89a"):
        return struct.unpack("<HH", b[6:10])
    return None


def _dims_jpeg(b: bytes):
    if b[:2] != b"\xff\xd8":
        return None
    i = 2
    while i + 9 < len(b):
        if b[i] != 0xFF:
            i += 1
            continue
        marker = b[i + 1]
        if marker in (0xD8, 0x01) or 0xD0 <= marker <= 0xD7:
            i += 2
            continue
        seg = struct.unpack(">H", b[i + 2:i + 4])[0]
        if marker in (0xC0, 0xC1, 0xC2, 0xC3, 0xC5, 0xC6, 0xC7, 0xC9, 0xCA, 0xCB, 0xCD, 0xCE, 0xCF):
            h, w = struct.unpack(">HH", b[i + 5:i + 9])
            return w, h
        i += 2 + seg
    return None


def _dims_webp(b: bytes):
    if b[:4] != b"RIFF" or b[8:12] != b"WEBP":
        return None
    kind = b[12:16]
    if kind == b"VP8X":
        w = 1 + int.from_bytes(b[24:27], "little")
        h = 1 + int.from_bytes(b[27:30], "little")
        return w, h
    if kind == b"VP8 " and b[23:26] == b"\x9d\x01\x2a":
        w, h = struct.unpack("<HH", b[26:30])
        return w & 0x3FFF, h & 0x3FFF
    if kind == b"VP8L" and b[20] == 0x2F:
        v = int.from_bytes(b[21:25], "little")
        return (v & 0x3FFF) + 1, ((v >> 14) & 0x3FFF) + 1
    return None


def image_dims(url: str) -> Optional[tuple[int, int]]:
    """(width, height) from a base64 data: URL header, None otherwise."""
    if not url.startswith("data:") or ";base64," not in url:
        return None
    try:
        head = base64.b64decode(url.split(";base64,", 1)[1][:4096] + "===", validate=False)
    except (ValueError, TypeError):
        return None
    for f in (_dims_png, _dims_jpeg, _dims_gif, _dims_webp):
        try:
            d = f(head)
        except (struct.error, IndexError):
            d = None
        if d:
            return int(d[0]), int(d[1])
    return None


@dataclass
class TokenEstimator:
    strategy: str = "dimension"   # dimension | fixed
    factor: int = 784
    fixed_tokens: int = 280

    @classmethod
    def from_params(cls, p: Optional[dict]) -> "TokenEstimator":
        p = p or {}
        return cls(p.get("strategy", "dimension"), int(p.get("factor", 784)), int(p.get("fixedTokens", 280)))

    def tokens(self, url: str) -> int:
        if self.strategy == "dimension":
            d = image_dims(url)
            if d:
                return max(1, math.ceil(d[0] * d[1] / self.factor))
        return self.fixed_tokens


def asset_hash(url: str) -> str:
    return hashlib.sha256(url.encode()).hexdigest()[:16]


def virtual_segment(url: str, est: TokenEstimator) -> str:
    """Deterministic placeholder of the image's estimated character footprint."""
    h = asset_hash(url)
    n = est.tokens(url) * CHARS_PER_TOKEN
    body = (h * (n // len(h) + 1))[:n]
    return f"<img:{h}>" + body


def image_url_of(part: dict) -> Optional[str]:
    if part.get("type") in ("image_url", "input_image"):
        iu = part.get("image_url")
        if isinstance(iu, dict):
            return iu.get("url")
        return iu if isinstance(iu, str) else part.get("url")
    return None
