"""Vision tower + multimodal Llama (the E in E/PD disaggregation; SURVEY C27,
reference guides/multimodal-serving/e-disaggregation/README.md:1-46).

Qwen2-VL-style dynamic-resolution encoder: the image is resized to a multiple
of ``patch * merge`` (14 * 2 = 28 px) within ``max_pixels``, cut into 14x14
patches, embedded by a linear patch projection + learned 2-D position
embedding, run through pre-LN transformer blocks (non-causal SDPA, one
image = one sequence), and every 2x2 patch group is merged and projected to
the LM hidden size. One image of W x H pixels -> (W/28)*(H/28) LM tokens,
the dimension strategy the router's multimodal scorer assumes (factor 784,
router/multimodal.py).

``MMInput`` ties those embeddings to the prompt: a run of ``image_token_id``
placeholders at ``offset`` of length ``length``. The model runner overwrites
the embedding rows of the placeholders inside each prefill chunk, so chunked
prefill, prefix caching (image hashes fold into the block-key ``extra``) and
P/D all work unchanged.
"""
from __future__ import annotations

import base64
import hashlib
import io
import math
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn.functional as F

from llmd_amd.engine.attn_meta import AttnMeta

from .layers import _init_weight
from .llama import LlamaForCausalLM

MEAN = (0.48145466, 0.4578275, 0.40821073)
STD = (0.26862954, 0.26130258, 0.27577711)


@dataclass
class VisionConfig:
    hidden_size: int = 1280
    num_layers: int = 32
    num_heads: int = 16
    mlp_ratio: float = 3.5
    patch_size: int = 14
    merge_size: int = 2
    max_pixels: int = 1280 * 28 * 28
    min_pixels: int = 4 * 28 * 28
    max_pos: int = 64  # position-embedding grid side (patches)


@dataclass
class MMInput:
    offset: int                      # first placeholder token position in the prompt
    length: int                      # number of placeholder tokens
    mm_hash: str                     # hex sha256 of the image bytes
    embeds: Optional[torch.Tensor] = None   # [length, d_model] bf16 (device or host)
    meta: dict = field(default_factory=dict)


# ---------------------------------------------------------------- image I/O
def load_image_bytes(url: str) -> bytes:
    """data: URLs (base64) and local file:// paths; there is no network access."""
    if url.startswith("data:"):
        head, _, data = url.partition(",")
        if ";base64" not in head:
            raise ValueError("only base64 data URLs are supported")
        return base64.b64decode(data)
    if url.startswith("file://"):
        with open(url[7:], "rb") as f:
            return f.read()
    raise ValueError("image_url must be a data: URL or file:// path (no remote fetch)")


def mm_hash(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def smart_resize(w: int, h: int, cfg: VisionConfig) -> tuple[int, int]:
    f = cfg.patch_size * cfg.merge_size
    W = max(f, round(w / f) * f)
    H = max(f, round(h / f) * f)
    if W * H > cfg.max_pixels:
        s = math.sqrt(w * h / cfg.max_pixels)
        W, H = max(f, math.floor(w / s / f) * f), max(f, math.floor(h / s / f) * f)
    elif W * H < cfg.min_pixels:
        s = math.sqrt(cfg.min_pixels / (w * h))
        W, H = math.ceil(w * s / f) * f, math.ceil(h * s / f) * f
    return W, H


def num_image_tokens(w: int, h: int, cfg: VisionConfig) -> int:
    W, H = smart_resize(w, h, cfg)
    f = cfg.patch_size * cfg.merge_size
    return (W // f) * (H // f)


def preprocess(b: bytes, cfg: VisionConfig) -> torch.Tensor:
    """Image bytes -> normalised float pixels [3, H, W] at the model resolution."""
    from PIL import Image

    im = Image.open(io.BytesIO(b)).convert("RGB")
    W, H = smart_resize(im.width, im.height, cfg)
    im = im.resize((W, H), Image.BICUBIC)
    x = torch.frombuffer(bytearray(im.tobytes()), dtype=torch.uint8).view(H, W, 3).permute(2, 0, 1).float() / 255
    m = torch.tensor(MEAN).view(3, 1, 1)
    s = torch.tensor(STD).view(3, 1, 1)
    return (x - m) / s


# ---------------------------------------------------------------- encoder
class _Block(torch.nn.Module):
    def __init__(self, d, heads, ratio, device, dt):
        super().__init__()
        self.heads = heads
        self.n1 = torch.nn.LayerNorm(d, device=device, dtype=dt)
        self.qkv = torch.nn.Linear(d, 3 * d, device=device, dtype=dt)
        self.proj = torch.nn.Linear(d, d, device=device, dtype=dt)
        self.n2 = torch.nn.LayerNorm(d, device=device, dtype=dt)
        f = int(d * ratio)
        self.fc1 = torch.nn.Linear(d, f, device=device, dtype=dt)
        self.fc2 = torch.nn.Linear(f, d, device=device, dtype=dt)

    def forward(self, x):  # x [N, d]
        N, d = x.shape
        q, k, v = self.qkv(self.n1(x)).view(N, 3, self.heads, d // self.heads).permute(1, 2, 0, 3)
        a = F.scaled_dot_product_attention(q, k, v)  # [heads, N, hd]
        x = x + self.proj(a.transpose(0, 1).reshape(N, d))
        return x + self.fc2(F.gelu(self.fc1(self.n2(x)), approximate="tanh"))


class VisionEncoder(torch.nn.Module):
    def __init__(self, cfg: VisionConfig, d_model: int, device="cuda", dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        d, p = cfg.hidden_size, cfg.patch_size
        self.patch = torch.nn.Linear(3 * p * p, d, bias=False, device=device, dtype=dtype)
        self.pos = torch.nn.Parameter(_init_weight(torch.empty(cfg.max_pos * cfg.max_pos, d, device=device,
                                                               dtype=dtype), 0.02), requires_grad=False)
        self.blocks = torch.nn.ModuleList(
            [_Block(d, cfg.num_heads, cfg.mlp_ratio, device, dtype) for _ in range(cfg.num_layers)])
        self.norm = torch.nn.LayerNorm(d, device=device, dtype=dtype)
        m2 = cfg.merge_size ** 2
        self.merge1 = torch.nn.Linear(d * m2, d * m2, device=device, dtype=dtype)
        self.merge2 = torch.nn.Linear(d * m2, d_model, device=device, dtype=dtype)
        for mod in self.modules():
            if isinstance(mod, torch.nn.Linear):
                _init_weight(mod.weight.data, 0.02)
                if mod.bias is not None:
                    mod.bias.data.zero_()
        for prm in self.parameters():
            prm.requires_grad_(False)

    @torch.no_grad()
    def forward(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [3, H, W] (H, W multiples of patch*merge) -> [H*W/(p*m)^2, d_model]."""
        cfg = self.cfg
        p, mg = cfg.patch_size, cfg.merge_size
        dev = self.patch.weight.device
        x = pixels.to(dev, self.patch.weight.dtype)
        _, H, W = x.shape
        gh, gw = H // p, W // p
        # patches ordered so every merge group (mg x mg) is contiguous
        x = x.view(3, gh // mg, mg, p, gw // mg, mg, p).permute(1, 4, 2, 5, 0, 3, 6).reshape(gh * gw, 3 * p * p)
        h = self.patch(x)
        iy = torch.arange(gh, device=dev).view(gh // mg, mg, 1, 1).expand(gh // mg, mg, gw // mg, mg)
        ix = torch.arange(gw, device=dev).view(1, 1, gw // mg, mg).expand(gh // mg, mg, gw // mg, mg)
        pos = ((iy.permute(0, 2, 1, 3) % cfg.max_pos) * cfg.max_pos + ix.permute(0, 2, 1, 3) % cfg.max_pos)
        h = h + self.pos[pos.reshape(-1)]
        for b in self.blocks:
            h = b(h)
        h = self.norm(h).reshape(-1, h.shape[1] * mg * mg)
        return self.merge2(F.gelu(self.merge1(h)))


class LlavaForCausalLM(LlamaForCausalLM):
    """Llama LM + vision tower. ``meta.mm_rows``/``meta.mm_embeds`` (set by the
    runner for prefill chunks that cover image placeholders) replace the
    placeholder embeddings."""

    def __init__(self, cfg, device="cuda", max_pos: int = 32768):
        super().__init__(cfg, device, max_pos)
        self.vision_cfg = VisionConfig(**(cfg.vision_config or {}))
        self.vision = VisionEncoder(self.vision_cfg, cfg.hidden_size, device)

    def encode_image(self, b: bytes) -> torch.Tensor:
        return self.vision(preprocess(b, self.vision_cfg))

    def forward(self, input_ids: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        x = self.embed(input_ids)
        rows = getattr(meta, "mm_rows", None)
        if rows is not None:
            x = x.index_copy(0, rows, meta.mm_embeds.to(x.dtype))
        residual = None
        for layer in self.layers:
            x, residual = layer(x, residual, meta)
        x, _ = self.norm(x, residual)
        return x


def chunk_mm_rows(mm: list[MMInput], start: int, n: int, row0: int):
    """Rows of a prefill chunk [start, start+n) (placed at step row ``row0``)
    that are image placeholders, with the matching embedding slices."""
    rows, embs = [], []
    for it in mm:
        lo, hi = max(it.offset, start), min(it.offset + it.length, start + n)
        if lo < hi and it.embeds is not None:
            rows.extend(range(row0 + lo - start, row0 + hi - start))
            embs.append(it.embeds[lo - it.offset:hi - it.offset])
    return rows, embs


def mm_cache_key(mm: list[MMInput]) -> int:
    """64-bit block-key namespace for a request's images (folded into `extra`)."""
    h = hashlib.sha256("".join(i.mm_hash for i in mm).encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 63) - 1)
