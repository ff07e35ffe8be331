"""Multimodal-aware prefix scoring (C28): image token estimation from data-URL
headers (dimension and fixed strategies) and its effect on approximate
prefix block keys."""
import base64
import json
import struct
import zlib

from llmd_amd import _rt_loader
from llmd_amd.router.multimodal import TokenEstimator, image_dims
from llmd_amd.router.plugins.parsers import OpenAIParser


def _png(w, h):
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)
    chunk = b"IHDR" + ihdr
    raw = b"\x89PNG\r\n\x1a\n" + struct.pack(">I", 13) + chunk + struct.pack(">I", zlib.crc32(chunk))
    return "data:image/png;base64," + base64.b64encode(raw + b"\x00" * 32).decode()


def _gif(w, h):
    return "data:image/gif;base64," + base64.b64encode(b"GIF89a" + struct.pack("<HH", w, h) + b"\x00" * 16).decode()


def _jpeg(w, h):
    sof = b"\xff\xc0" + struct.pack(">HBHH", 17, 8, h, w) + b"\x03" + b"\x00" * 9
    raw = b"\xff\xd8" + b"\xff\xe0" + struct.pack(">H", 16) + b"JFIF\x00" + b"\x00" * 9 + sof
    return "data:image/jpeg;base64," + base64.b64encode(raw).decode()


def test_image_dims_and_estimates():
    assert image_dims(_png(448, 448)) == (448, 448)
    assert image_dims(_gif(640, 480)) == (640, 480)
    assert image_dims(_jpeg(1024, 768)) == (1024, 768)
    assert image_dims("https://example.com/cat.png") is None
    qwen25 = TokenEstimator("dimension", 784)
    assert qwen25.tokens(_png(448, 448)) == 256
    assert TokenEstimator("dimension", 1024).tokens(_png(448, 448)) == 196
    assert qwen25.tokens("https://x/y.jpg") == 280                    # unknown dims -> fixed
    assert TokenEstimator("fixed", fixed_tokens=560).tokens(_png(32, 32)) == 560


def _chat(img, text="what is this"):
    return json.dumps({"model": "m", "messages": [{"role": "user", "content": [
        {"type": "image_url", "image_url": {"url": img}}, {"type": "text", "text": text}]}]}).encode()


def test_parser_virtual_segments_drive_prefix_blocks():
    p = OpenAIParser("openai-parser", {"multimodal": {"strategy": "dimension", "factor": 784}})
    a = p.parse("/v1/chat/completions", _chat(_png(448, 448)), {})
    b = p.parse("/v1/chat/completions", _chat(_png(448, 448), "other question"), {})
    c = p.parse("/v1/chat/completions", _chat(_png(224, 224)), {})
    assert a.mm_assets and a.mm_assets[0][1] == 256
    rt = _rt_loader.rt()
    ka = rt.char_block_hashes(a.prompt, 64, 0, 1000)
    kb = rt.char_block_hashes(b.prompt, 64, 0, 1000)
    kc = rt.char_block_hashes(c.prompt, 64, 0, 1000)
    # ~256 tokens of image footprint -> >= 16 shared 64-char blocks for the same image
    shared_ab = next((i for i, (x, y) in enumerate(zip(ka, kb)) if x != y), min(len(ka), len(kb)))
    assert shared_ab >= 16
    assert ka[0] != kc[0]  # a different image diverges immediately
