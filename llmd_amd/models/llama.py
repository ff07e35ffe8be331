"""Llama-family decoder (Llama-3 8B/70B, Qwen3 dense) on the paged-KV engine.

Per layer (dense TP=k):
  fused_add_rmsnorm -> QKV GEMM -> rope+cache write -> paged attention
  -> O GEMM (+TP all-reduce) -> fused_add_rmsnorm -> gate_up GEMM
  -> SiLU*mul -> down GEMM (+TP all-reduce)
Residual stream is carried separately so every norm fuses the residual add.
Decode steps on the split-K medium-M GEMM (csrc/ops/mgemm.hip) fold the
kernels after each projection into its reduce: QKV reduce + RoPE + cache write
(rope_cache.hip reduce_rope_cache_kernel), o / down reduce + residual add +
the next RMSNorm (mgemm_reduce_norm_kernel), bit-identical to the unfused path.
"""
from __future__ import annotations

from typing import Optional

import torch

from llmd_amd import ops
from llmd_amd.engine.attn_meta import AttnMeta
from llmd_amd.engine.config import ModelConfig
from llmd_amd.parallel.state import get_state

from .layers import ColumnLinear, LMHead, PagedAttention, RMSNorm, RowLinear, VocabEmbedding, wants_fp8_input


class LlamaMLP(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, device):
        super().__init__()
        self.gate_up = ColumnLinear(cfg.hidden_size, 2 * cfg.intermediate_size, device=device)
        self.down = RowLinear(cfg.intermediate_size, cfg.hidden_size, device=device)

    def forward(self, x):
        return self.down(self.hidden(x))

    def hidden(self, x):
        """silu(x Wg^T) * (x Wu^T): the down projection's input (fp8 (q, scale) for an fp8 down)."""
        gu = self.gate_up
        if (gu.lora is None and gu.bias is None and not wants_fp8_input(self.down) and x.dim() == 2
                and gu.weight.dtype == torch.bfloat16):
            # prefill: gate/up GEMM with the SiLU-and-mul in its epilogue (csrc/ops/pgemm.hip
            # EPI_SILU_STD) where the shipped table has it ahead of hipBLASLt + the act kernel
            v = ops.pgemm_silu_plan(x, gu.weight)
            if v is not None:
                return ops.pgemm_silu(x, gu.weight, variant=v)
            # decode: the same fusion in the medium-M GEMM (csrc/ops/mgemm.hip ACT form)
            p = ops.mgemm_silu_plan(x, gu.weight)
            if p is not None:
                return ops.mgemm_silu(x, gu.weight, p)
        x0 = x[0] if isinstance(x, tuple) else x
        if (wants_fp8_input(self.down) and wants_fp8_input(gu) and gu.bias is None and x0.dim() == 2
                and ops._gpu(x0) and ops.pgemm8_silu_planned(x0.shape[0], gu.weight.shape[0], gu.weight.shape[1])):
            # fp8 prefill: SiLU-and-mul in the fp8 gate/up GEMM's epilogue (csrc/ops/pgemm8.hip), then
            # the per-token quant of the [M, F] activation (half the bytes of the act-quant's input)
            xq, xs = x if isinstance(x, tuple) else ops.quant_fp8_rows(x)
            if ops.pgemm_fp8_ok(xq, gu.weight):
                return ops.quant_fp8_rows(ops.pgemm_fp8(xq, xs, gu.weight, gu.weight_scale, epi=3))
        h = gu(x)
        if wants_fp8_input(self.down):  # SiLU*up fused with the down proj's fp8 activation quant
            return ops.gated_act_quant(h, ops.ACT_SILU)
        return ops.gated_act(h, ops.ACT_SILU)


def qkv_fused_plan(lin, x):
    """Medium-M GEMM plan of the QKV projection when its split-K reduce can be fused with RoPE + the
    cache write (ops.reduce_rope_cache), or None: bf16 weights without bias or LoRA, decode-sized M,
    a shipped plan that splits K."""
    if (not isinstance(x, torch.Tensor) or lin.bias is not None or lin.lora is not None
            or lin.weight.dtype != torch.bfloat16 or not (ops.MGEMM_NORM and ops._SKINNY)
            or lin.weight.shape[0] > 24576):
        return None
    if not (x.dim() == 2 and 33 <= x.shape[0] <= 128 and ops.mgemm_ok(x, lin.weight)):
        return None
    plan = ops.mgemm_choice(x.shape[0], lin.weight.shape[0], lin.weight.shape[1])
    return plan if plan is not None and plan[1] >= 2 and lin.weight.shape[1] // 64 >= 2 else None


def norm_fused_plan(lin, x):
    """Medium-M GEMM plan for ``lin(x)`` with the following residual-add + RMSNorm fused into its
    split-K reduce (ops.mgemm_add_rmsnorm), or None: bf16 TP1 row-parallel linears without bias or
    LoRA at decode-sized M (33..128) whose shipped plan splits K."""
    if (not isinstance(x, torch.Tensor) or lin.bias is not None or lin.lora is not None
            or lin.weight.dtype != torch.bfloat16 or (lin.reduce and get_state().tp_size > 1)):
        return None
    return ops.mgemm_norm_plan(x, lin.weight)


class LlamaDecoderLayer(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, idx: int, cos_sin: torch.Tensor, device):
        super().__init__()
        d, D = cfg.hidden_size, cfg.head_dim
        Hq, Hkv = cfg.num_attention_heads, cfg.num_key_value_heads
        self.cfg = cfg
        self.input_layernorm = RMSNorm(d, cfg.rms_norm_eps, device)
        self.qkv = ColumnLinear(d, (Hq + 2 * Hkv) * D, bias=cfg.attention_bias, device=device)
        self.attn = PagedAttention(idx, Hq, Hkv, D, cos_sin, window=cfg.layer_window(idx),
                                   sinks=cfg.attention_sinks, device=device)
        self.o_proj = RowLinear(Hq * D, d, bias=cfg.attention_bias and cfg.model_type == "gpt_oss", device=device)
        self.post_attention_layernorm = RMSNorm(d, cfg.rms_norm_eps, device)
        self.mlp = self._make_mlp(cfg, idx, device)
        # Qwen3: per-head RMSNorm on q and k before rope
        self.qk_norm = cfg.model_type in ("qwen3", "qwen3_moe")
        if self.qk_norm:
            self.q_norm = RMSNorm(D, cfg.rms_norm_eps, device)
            self.k_norm = RMSNorm(D, cfg.rms_norm_eps, device)

    def _make_mlp(self, cfg, idx, device):
        return LlamaMLP(cfg, device)

    def _apply_qk_norm(self, qkv):
        a = self.attn
        ops.qk_rms_norm(qkv, self.q_norm.weight, self.k_norm.weight, a.Hq, a.Hkv, self.q_norm.eps)

    def forward(self, x, residual, meta: AttnMeta):
        x, residual, _ = self.run(x, residual, meta)
        return x, residual

    def run(self, x, residual, meta: AttnMeta, normed: bool = False, next_norm: Optional[RMSNorm] = None):
        """The layer with decode-step norm fusions. ``normed``: x already is this layer's
        input_layernorm output (fused into the previous layer's down projection). ``next_norm``:
        the RMSNorm that follows this layer (the next layer's input norm or the model's final
        norm); where the decode GEMM plan allows, the down projection's split-K reduce applies
        it and the third return value is True. The o projection always takes the
        post-attention norm this way when it can (csrc/ops/mgemm.hip mgemm_reduce_norm_kernel:
        bit-identical to GEMM + reduce + fused_add_rms_norm, two launches fewer)."""
        # W8A8: the norms emit fp8 + per-row scales straight into the fp8 GEMMs
        q_in = wants_fp8_input(self.qkv)
        if normed:
            pass
        elif residual is None:
            residual = x.clone()
            x = self.input_layernorm(x, quant=q_in)
        else:
            x, residual = self.input_layernorm(x, residual, quant=q_in)
        p = None if (self.qk_norm or q_in) else qkv_fused_plan(self.qkv, x)
        if p is not None:  # decode: the QKV split-K reduce fused with RoPE + the cache write
            parts = ops.mgemm_partials(x, self.qkv.weight, p)
            a = self.attn(torch.empty(x.shape[0], self.qkv.weight.shape[0], dtype=x.dtype, device=x.device), meta,
                          parts=parts)
        else:
            qkv = self.qkv(x)
            if self.qk_norm:
                self._apply_qk_norm(qkv)
            a = self.attn(qkv, meta)
        q_mlp = isinstance(self.mlp, LlamaMLP) and wants_fp8_input(self.mlp.gate_up)
        p = None if q_mlp else norm_fused_plan(self.o_proj, a)
        if p is not None:
            pn = self.post_attention_layernorm
            x = ops.mgemm_add_rmsnorm(a, self.o_proj.weight, p, residual, pn.weight, pn.eps)
        else:
            x = self.o_proj(a)
            x, residual = self.post_attention_layernorm(x, residual, quant=q_mlp)
        if next_norm is not None and type(self.mlp) is LlamaMLP:
            h = self.mlp.hidden(x)
            p = norm_fused_plan(self.mlp.down, h)
            if p is not None:
                return ops.mgemm_add_rmsnorm(h, self.mlp.down.weight, p, residual, next_norm.weight,
                                             next_norm.eps), residual, True
            return self.mlp.down(h), residual, False
        return self.mlp(x), residual, False


class LlamaForCausalLM(torch.nn.Module):
    layer_cls = LlamaDecoderLayer

    def __init__(self, cfg: ModelConfig, device="cuda", max_pos: int = 32768):
        super().__init__()
        self.cfg = cfg
        rot = cfg.head_dim
        self.register_buffer("cos_sin", ops.rope_cos_sin(rot, max_pos, cfg.rope_theta, cfg.rope_scaling,
                                                         device=device), persistent=False)
        self.embed = VocabEmbedding(cfg.vocab_size, cfg.hidden_size, device)
        self.layers = torch.nn.ModuleList(
            [self.layer_cls(cfg, i, self.cos_sin, device) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, device)
        self.lm_head = LMHead(cfg.vocab_size, cfg.hidden_size, device,
                              tied=self.embed if cfg.tie_word_embeddings else None)

    def attention_layers(self):
        return [layer.attn for layer in self.layers]

    def weight_specs(self) -> list:
        """HF checkpoint names -> this rank's parameters (models/loader.py)."""
        cfg = self.cfg
        D, Hq, Hkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads
        specs = [("model.embed_tokens.weight", self.embed.weight, "vocab", None),
                 ("model.norm.weight", self.norm.weight, "replicate", None)]
        if not cfg.tie_word_embeddings:
            specs.append(("lm_head.weight", self.lm_head.weight, "vocab", None))
        for i, layer in enumerate(self.layers):
            pre = f"model.layers.{i}."
            a = layer.attn
            q_rows, kv_rows = a.Hq * D, a.Hkv * D
            specs += [(pre + "input_layernorm.weight", layer.input_layernorm.weight, "replicate", None),
                      (pre + "post_attention_layernorm.weight", layer.post_attention_layernorm.weight,
                       "replicate", None),
                      (pre + "self_attn.o_proj.weight", layer.o_proj.weight, "row", None)]
            for nm, off, nh in (("q_proj", 0, Hq), ("k_proj", q_rows, Hkv), ("v_proj", q_rows + kv_rows, Hkv)):
                specs.append((pre + f"self_attn.{nm}.weight", layer.qkv.weight, "fused", (off, nh, D)))
                if layer.qkv.bias is not None:
                    specs.append((pre + f"self_attn.{nm}.bias", layer.qkv.bias, "fused", (off, nh, D)))
            if layer.o_proj.bias is not None:
                specs.append((pre + "self_attn.o_proj.bias", layer.o_proj.bias, "replicate", None))
            if layer.qk_norm:
                specs += [(pre + "self_attn.q_norm.weight", layer.q_norm.weight, "replicate", None),
                          (pre + "self_attn.k_norm.weight", layer.k_norm.weight, "replicate", None)]
            if a.sinks is not None:
                specs.append((pre + "self_attn.sinks", a.sinks, "col", None))
            specs += self._mlp_specs(pre, layer.mlp)
        return specs

    def _mlp_specs(self, pre: str, mlp) -> list:
        F_total = self.cfg.intermediate_size
        F_local = mlp.gate_up.weight.shape[0] // 2
        return [(pre + "mlp.gate_proj.weight", mlp.gate_up.weight, "fused", (0, F_total, 1)),
                (pre + "mlp.up_proj.weight", mlp.gate_up.weight, "fused", (F_local, F_total, 1)),
                (pre + "mlp.down_proj.weight", mlp.down.weight, "row", None)]

    @torch.no_grad()
    def forward(self, input_ids: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        x = self.embed(input_ids)
        residual = None
        normed = False
        n = len(self.layers)
        for i, layer in enumerate(self.layers):
            if not isinstance(layer, LlamaDecoderLayer) or type(layer).forward is not LlamaDecoderLayer.forward:
                x, residual = layer(x, residual, meta)
                normed = False
                continue
            # the norm after this layer, for the decode down projection's fused reduce
            nxt = self.layers[i + 1] if i + 1 < n else None
            if nxt is None:
                nn = self.norm
            elif (isinstance(nxt, LlamaDecoderLayer) and type(nxt).forward is LlamaDecoderLayer.forward
                  and not wants_fp8_input(nxt.qkv)):
                nn = nxt.input_layernorm
            else:
                nn = None
            x, residual, normed = layer.run(x, residual, meta, normed, nn)
        if normed:
            return x
        x, _ = self.norm(x, residual)
        return x

    @torch.no_grad()
    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        return self.lm_head(h)


def kv_head_count(cfg: ModelConfig) -> int:
    return max(1, cfg.num_key_value_heads // get_state().tp_size)
