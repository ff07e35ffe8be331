"""Model building blocks: TP-sharded linears, norms, embeddings, paged attention.

Weights are plain bf16 tensors in [out, in] layout and GEMMs go to hipBLASLt
through ``torch.nn.functional.linear`` ("hipBLASLt first").
Fused elementwise work (norm + residual, rope + cache write, gated activation)
runs in the hand-written HIP kernels of ``llmd_amd.ops``.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from llmd_amd import ops
from llmd_amd.engine.attn_meta import AttnMeta
from llmd_amd.parallel.comm import tp_all_gather, tp_all_reduce
from llmd_amd.parallel.state import get_state


def _init_weight(t: torch.Tensor, std: float, gen: Optional[torch.Generator] = None):
    with torch.no_grad():
        if t.is_cuda:
            t.normal_(0.0, std, generator=gen)
        else:
            t.copy_(torch.randn(t.shape, generator=gen) * std)
    return t


def _linear(mod, x, bias):
    """bf16 weights -> hipBLASLt GEMM, or the decode GEMM kernel for the decode
    shapes where it measured faster (ops.linear); fp8 weights (quantize_fp8) ->
    W8A8 GEMM with dynamic per-token activation scales."""
    w = mod.weight
    if w.dtype == torch.float8_e4m3fn:
        return ops.fp8_linear(x, w, mod.weight_scale, bias)
    return ops.linear(x, w, bias)


def wants_fp8_input(lin) -> bool:
    """A linear that can consume a pre-quantised (q, scale) activation."""
    return lin.weight.dtype == torch.float8_e4m3fn and lin.lora is None


def quantize_fp8(model: torch.nn.Module) -> int:
    """Online FP8 weight quantisation (vLLM ``--quantization fp8``): every
    Column/Row linear gets e4m3fn weights with per-output-channel scales, and
    routed-expert weights (modules with 3-D ``w1``/``w2``) get DeepSeek-style
    128x128 block scales for the fp8 grouped GEMM. Embeddings, LM head, norms
    and routers stay bf16. Returns the number of quantised tensors."""
    n = 0
    for m in model.modules():
        if isinstance(m, (ColumnLinear, RowLinear)) and m.weight.dtype == torch.bfloat16:
            wq, s = ops.quant_fp8_weight(m.weight.data)
            m.weight = torch.nn.Parameter(wq, requires_grad=False)
            m.weight_scale = torch.nn.Parameter(s, requires_grad=False)
            n += 1
        for name in ("w1", "w2"):
            w = getattr(m, name, None)
            if isinstance(w, torch.Tensor) and w.dim() == 3 and w.dtype == torch.bfloat16:
                wq, s = ops.quant_fp8_block_weight(w.data)
                if w.is_cuda and w.shape[2] % 128:  # whole 128-wide K-steps for the v2 grouped GEMM
                    wq = ops.pad_fp8_k(wq, (w.shape[2] + 127) // 128 * 128)
                setattr(m, name, torch.nn.Parameter(wq, requires_grad=False))
                setattr(m, name + "_scale", torch.nn.Parameter(s, requires_grad=False))
                n += 1
    return n


def quantize_mxfp4(model: torch.nn.Module) -> int:
    """``--quantization mxfp4``: routed-expert weights in OCP MXFP4 (e2m1 codes + E8M0 scale per 32
    elements - the format gpt-oss's checkpoint ships its experts in; vLLM's mxfp4 method), K padded
    to a multiple of 128 and to >= 512 (the persistent tile kernel peels its last 3 K-steps); every
    Column/Row linear takes the fp8 W8A8 path of quantize_fp8 (no MXFP4 kernel for those GEMMs). Returns the number of quantised tensors."""
    n = 0
    for m in model.modules():
        for name in ("w1", "w2"):
            w = getattr(m, name, None)
            if isinstance(w, torch.Tensor) and w.dim() == 3 and w.dtype == torch.bfloat16:
                kp = max(512, (w.shape[2] + 127) // 128 * 128)
                q, s = ops.quant_mxfp4_weight(ops.pad_mxfp4_k(w.data, kp))
                # K-step major codes and scales: contiguous weight DMA per K-step
                q, s = ops.mxfp4_kernel_layout(q), ops.mxfp4_scales_kernel_layout(s)
                setattr(m, name, torch.nn.Parameter(q, requires_grad=False))
                setattr(m, name + "_scale", torch.nn.Parameter(s, requires_grad=False))
                n += 1
    return n + quantize_fp8(model)


def is_mxfp4_experts(mod) -> bool:
    return mod.w1.dtype == torch.uint8 and getattr(mod, "w1_scale", None) is not None


def run_experts(mod, x, ids, w, act, alpha=1.702, limit=7.0, b1=None, b2=None):
    """Routed-expert FFN of an MoE module: bf16, block-fp8 or MXFP4 grouped GEMMs."""
    if is_mxfp4_experts(mod):
        return ops.moe_experts_mxfp4(x, ids, w, mod.w1, mod.w1_scale, mod.w2, mod.w2_scale, act, alpha, limit,
                                     b1=b1, b2=b2)
    if mod.w1.dtype == torch.float8_e4m3fn:
        return ops.moe_experts_fp8(x, ids, w, mod.w1, mod.w1_scale, mod.w2, mod.w2_scale, act, alpha, limit,
                                   b1=b1, b2=b2)
    if isinstance(x, ops.Fp8Rows):
        x = x.dequant()
    return ops.moe_experts(x, ids, w, mod.w1, mod.w2, act, alpha, limit, b1=b1, b2=b2)


class ColumnLinear(torch.nn.Module):
    """y = x W^T, W [out/tp, in]; output stays sharded."""

    def __init__(self, in_f: int, out_f: int, bias=False, device=None, dtype=torch.bfloat16,
                 shard=True, std=0.02):
        super().__init__()
        tp = get_state().tp_size if shard else 1
        assert out_f % tp == 0, (out_f, tp)
        self.in_f, self.out_f = in_f, out_f // tp
        self.weight = torch.nn.Parameter(_init_weight(torch.empty(self.out_f, in_f, device=device, dtype=dtype), std),
                                         requires_grad=False)
        self.bias = torch.nn.Parameter(torch.zeros(self.out_f, device=device, dtype=dtype),
                                       requires_grad=False) if bias else None

    lora = None  # engine/lora.py LoRATarget when multi-LoRA is enabled

    def forward(self, x):
        y = _linear(self, x, self.bias)
        if self.lora is not None:
            self.lora.apply(y, x)
        return y


class RowLinear(torch.nn.Module):
    """y = all_reduce(x_shard W_shard^T), W [out, in/tp]."""

    def __init__(self, in_f: int, out_f: int, bias=False, device=None, dtype=torch.bfloat16,
                 reduce=True, std=0.02):
        super().__init__()
        tp = get_state().tp_size
        assert in_f % tp == 0
        self.in_f, self.out_f, self.reduce = in_f // tp, out_f, reduce
        self.weight = torch.nn.Parameter(_init_weight(torch.empty(out_f, self.in_f, device=device, dtype=dtype), std),
                                         requires_grad=False)
        self.bias = torch.nn.Parameter(torch.zeros(out_f, device=device, dtype=dtype),
                                       requires_grad=False) if bias else None

    lora = None

    def forward(self, x):
        # one rank (no reduce to follow): the bias rides in the GEMM epilogue instead of a separate add
        fold = self.bias is not None and self.lora is None and (not self.reduce or get_state().tp_size == 1)
        y = _linear(self, x, self.bias if fold else None)
        if self.lora is not None:  # partial sums join the layer's all-reduce
            self.lora.apply(y, x)
        if self.reduce:
            y = tp_all_reduce(y)
        if self.bias is not None and not fold:
            y = y + self.bias
        return y


class RMSNorm(torch.nn.Module):
    def __init__(self, d: int, eps: float, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(d, device=device, dtype=dtype), requires_grad=False)

    def forward(self, x, residual: Optional[torch.Tensor] = None, quant: bool = False):
        """quant=True: emit (fp8 q, per-row scale) for a W8A8 consumer (fused K05 + K16)."""
        if quant:
            q = ops.rms_norm_quant(x, self.weight, self.eps, residual)
            return q if residual is None else (q, residual)
        if residual is None:
            return ops.rms_norm(x, self.weight, self.eps)
        ops.fused_add_rms_norm(x, residual, self.weight, self.eps)
        return x, residual


class VocabEmbedding(torch.nn.Module):
    """Vocab-parallel embedding: each TP rank holds a vocab slice."""

    def __init__(self, vocab: int, d: int, device=None, dtype=torch.bfloat16):
        super().__init__()
        st = get_state()
        self.tp, self.rank = st.tp_size, st.tp_rank
        self.vocab = vocab
        # padded to 64 rows: logits rows stay 16-B aligned for the sampling kernel (odd vocabs, e.g. +1 image token)
        self.per = math.ceil(math.ceil(vocab / self.tp) / 64) * 64
        self.lo = self.rank * self.per
        self.weight = torch.nn.Parameter(_init_weight(torch.empty(self.per, d, device=device, dtype=dtype), 0.02),
                                         requires_grad=False)

    def forward(self, ids):
        if self.tp == 1:
            return F.embedding(ids, self.weight)
        local = ids - self.lo
        mask = (local < 0) | (local >= self.per)
        out = F.embedding(local.clamp(0, self.per - 1), self.weight)
        out.masked_fill_(mask[:, None], 0)
        return tp_all_reduce(out)


class LMHead(torch.nn.Module):
    def __init__(self, vocab: int, d: int, device=None, dtype=torch.bfloat16, tied: Optional[VocabEmbedding] = None):
        super().__init__()
        st = get_state()
        self.tp = st.tp_size
        self.vocab = vocab
        # padded to 64 rows: logits rows stay 16-B aligned for the sampling kernel (odd vocabs, e.g. +1 image token)
        self.per = math.ceil(math.ceil(vocab / self.tp) / 64) * 64
        if tied is not None:
            self.weight = tied.weight
        else:
            self.weight = torch.nn.Parameter(_init_weight(torch.empty(self.per, d, device=device, dtype=dtype), 0.02),
                                             requires_grad=False)

    def forward(self, h):
        logits = F.linear(h, self.weight)
        if self.tp > 1:
            logits = tp_all_gather(logits, -1)
        return logits[:, : self.vocab]


_ATTN_OVERLAP = os.environ.get("LLMD_ATTN_OVERLAP", "1") == "1"
_SIDE_STREAMS: dict = {}


def _overlap_stream(t: torch.Tensor):
    """The per-device side stream of mixed-step attention, or None (off, CPU, or under graph capture)."""
    if not (_ATTN_OVERLAP and t.is_cuda) or torch.cuda.is_current_stream_capturing():
        return None
    s = _SIDE_STREAMS.get(t.device.index)
    if s is None:
        s = _SIDE_STREAMS[t.device.index] = torch.cuda.Stream(device=t.device)
    return s


class PagedAttention(torch.nn.Module):
    """QKV projection output -> rope + cache write -> decode/prefill attention."""

    def __init__(self, layer_idx: int, num_heads: int, num_kv_heads: int, head_dim: int,
                 rope_cos_sin: torch.Tensor, window: int = 0, sinks: bool = False, neox: bool = True,
                 device=None):
        super().__init__()
        tp = get_state().tp_size
        assert num_heads % tp == 0
        self.layer_idx = layer_idx
        self.Hq = num_heads // tp
        self.Hkv = max(1, num_kv_heads // tp)
        self.D = head_dim
        self.scale = head_dim ** -0.5
        self.window = window
        self.neox = neox
        self.cos_sin = rope_cos_sin
        self.sinks = torch.nn.Parameter(torch.zeros(self.Hq, device=device, dtype=torch.float32),
                                        requires_grad=False) if sinks else None
        self.k_cache: Optional[torch.Tensor] = None
        self.v_cache: Optional[torch.Tensor] = None
        # fp8 KV dequant scales (checkpoint `self_attn.{k,v}_scale`; 1.0 otherwise)
        self.k_scale = 1.0
        self.v_scale = 1.0

    def forward(self, qkv: torch.Tensor, meta: AttnMeta, parts=None) -> torch.Tensor:
        """``parts`` = (fp32 split-K partials, nsplit) of the QKV projection whose reduce is fused
        with RoPE + the cache write (``qkv`` is then the allocated, unwritten output)."""
        T = qkv.shape[0]
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        if self.window and meta.swa is not None:  # hybrid KV cache: this layer's pool has its own tables
            meta = meta.swa
        if parts is not None:
            ops.reduce_rope_cache(parts[0], parts[1], qkv, meta.positions, self.cos_sin, Hq, Hkv, D,
                                  meta.slot_mapping, self.k_cache, self.v_cache, self.neox, self.k_scale,
                                  self.v_scale)
        else:
            ops.rope_cache(qkv, meta.positions, self.cos_sin, Hq, Hkv, D, meta.slot_mapping,
                           self.k_cache, self.v_cache, self.neox, self.k_scale, self.v_scale)
        out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
        nd = meta.num_decode
        # a mixed step (eager): the memory-bound decode rows run on a side stream beside the compute-bound
        # prefill attention (the decode kernel streams the running sequences' KV while the prefill's
        # MFMAs run; back to back they serialise)
        side = _overlap_stream(qkv) if nd and meta.num_prefill_tokens else None
        if nd:
            if side is not None:
                side.wait_stream(torch.cuda.current_stream(qkv.device))
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                ops.paged_decode(qkv[:nd], self.k_cache, self.v_cache, meta.d_block_tables,
                                 meta.d_seq_lens, Hq, Hkv, D, self.scale, self.window, self.sinks,
                                 split=meta.d_split, out=out[:nd], workspace=meta.d_workspace,
                                 max_ctx=meta.d_max_ctx, k_scale=self.k_scale, v_scale=self.v_scale,
                                 cascade=meta.d_cascade, split_dev=meta.d_split_dev)
        if meta.num_prefill_tokens:
            items = meta.p_items
            ops.paged_prefill(qkv[nd:], self.k_cache, self.v_cache, meta.p_block_tables,
                              meta.p_q_start, meta.p_q_len, meta.p_ctx_len, Hq, Hkv, D, self.scale,
                              self.window, self.sinks, items=items, out=out[nd:], k_scale=self.k_scale,
                              v_scale=self.v_scale)
        if side is not None:
            torch.cuda.current_stream(qkv.device).wait_stream(side)
        return out
