"""OPT decoder (facebook/opt-*) on the paged-KV engine.

OPT-125m is the model of the reference's CPU optimized-baseline path
(BASELINE config 1; ``docker/Dockerfile.cpu`` serves it through vLLM-CPU and
the router e2e scripts ``.github/scripts/e2e/`` drive it). Architecture (HF
``OPTForCausalLM``): learned absolute positions with an offset of 2, LayerNorm
with bias, biased q/k/v/out projections, a ReLU MLP (fc1 -> fc2), the LM head
tied to the token embedding, optional project_in/project_out when
``word_embed_proj_dim != hidden_size`` (opt-350m), pre-LN except opt-350m.

Per pre-LN layer (same engine contract as models/llama.py):
  fused residual-add + LayerNorm (csrc/ops/rmsnorm.hip layernorm_kernel)
  -> QKV GEMM (+bias) -> paged KV write (rope_cache with a zero-angle table:
  OPT has no rotary, the kernel only stores K/V) -> paged attention
  -> out GEMM (+bias, TP all-reduce) -> fused add + LayerNorm
  -> fc1 GEMM with bias + ReLU in the hipBLASLt epilogue (_addmm_activation)
  -> fc2 GEMM (+bias, TP all-reduce)
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from llmd_amd import ops
from llmd_amd.engine.attn_meta import AttnMeta
from llmd_amd.engine.config import ModelConfig

from .layers import ColumnLinear, LMHead, PagedAttention, RowLinear, VocabEmbedding, _init_weight

POS_OFFSET = 2  # HF OPTLearnedPositionalEmbedding


class LayerNorm(torch.nn.Module):
    def __init__(self, d: int, eps: float, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(d, device=device, dtype=dtype), requires_grad=False)
        self.bias = torch.nn.Parameter(torch.zeros(d, device=device, dtype=dtype), requires_grad=False)

    def forward(self, x, residual: Optional[torch.Tensor] = None):
        if residual is None:
            return ops.layer_norm(x, self.weight, self.bias, self.eps)
        ops.fused_add_layer_norm(x, residual, self.weight, self.bias, self.eps)
        return x, residual


def zero_angle_table(dim: int, max_pos: int, device) -> torch.Tensor:
    """[max_pos, dim] cos|sin table of angle 0: the rope+cache kernel leaves
    q/k unchanged and only writes K/V into the paged cache."""
    t = torch.zeros(max_pos, dim, dtype=torch.float32, device=device)
    t[:, : dim // 2] = 1.0
    return t


class OPTMLP(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, device):
        super().__init__()
        self.fc1 = ColumnLinear(cfg.hidden_size, cfg.intermediate_size, bias=cfg.attention_bias, device=device)
        self.fc2 = RowLinear(cfg.intermediate_size, cfg.hidden_size, bias=cfg.attention_bias, device=device)
        self.act = cfg.hidden_act

    def forward(self, x):
        f = self.fc1
        if self.act == "relu" and f.bias is not None and f.weight.dtype == torch.bfloat16 and f.lora is None:
            h = torch._addmm_activation(f.bias, x, f.weight.t())  # bias + ReLU fused into the GEMM epilogue
        else:
            h = f(x)
            h = F.relu(h) if self.act == "relu" else F.gelu(h)
        return self.fc2(h)


class OPTDecoderLayer(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, idx: int, cos_sin: torch.Tensor, device):
        super().__init__()
        d, D, H = cfg.hidden_size, cfg.head_dim, cfg.num_attention_heads
        self.pre_ln = cfg.do_layer_norm_before
        self.self_attn_layer_norm = LayerNorm(d, cfg.rms_norm_eps, device)
        self.qkv = ColumnLinear(d, 3 * H * D, bias=cfg.attention_bias, device=device)
        self.attn = PagedAttention(idx, H, H, D, cos_sin, device=device)
        self.out_proj = RowLinear(H * D, d, bias=cfg.attention_bias, device=device)
        self.final_layer_norm = LayerNorm(d, cfg.rms_norm_eps, device)
        self.mlp = OPTMLP(cfg, device)

    def forward(self, x, residual, meta: AttnMeta):
        if not self.pre_ln:  # opt-350m: LayerNorm after each residual add; the LN output is the residual
            h = self.out_proj(self.attn(self.qkv(x), meta))
            h, _ = self.self_attn_layer_norm(h, x)
            y = self.mlp(h)
            y, _ = self.final_layer_norm(y, h)
            return y, None
        if residual is None:
            residual = x.clone()
            x = self.self_attn_layer_norm(x)
        else:
            x, residual = self.self_attn_layer_norm(x, residual)
        x = self.out_proj(self.attn(self.qkv(x), meta))
        x, residual = self.final_layer_norm(x, residual)
        return self.mlp(x), residual


class OPTForCausalLM(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, device="cuda", max_pos: int = 32768):
        super().__init__()
        self.cfg = cfg
        d = cfg.hidden_size
        pd = cfg.word_embed_proj_dim or d
        self.register_buffer("cos_sin", zero_angle_table(cfg.head_dim, max_pos, device), persistent=False)
        self.embed = VocabEmbedding(cfg.vocab_size, pd, device)
        self.pos = torch.nn.Parameter(
            _init_weight(torch.empty(cfg.max_position_embeddings + POS_OFFSET, d, device=device,
                                     dtype=torch.bfloat16), 0.02), requires_grad=False)
        self.project_in = ColumnLinear(pd, d, shard=False, device=device) if pd != d else None
        self.project_out = ColumnLinear(d, pd, shard=False, device=device) if pd != d else None
        self.layers = torch.nn.ModuleList(
            [OPTDecoderLayer(cfg, i, self.cos_sin, device) for i in range(cfg.num_hidden_layers)])
        self.norm = LayerNorm(d, cfg.rms_norm_eps, device) if cfg.do_layer_norm_before else None
        self.lm_head = LMHead(cfg.vocab_size, pd, device, tied=self.embed if cfg.tie_word_embeddings else None)

    def attention_layers(self):
        return [layer.attn for layer in self.layers]

    def weight_specs(self) -> list:
        """HF checkpoint names -> this rank's parameters (models/loader.py)."""
        cfg = self.cfg
        D, H = cfg.head_dim, cfg.num_attention_heads
        p = "model.decoder."
        specs = [(p + "embed_tokens.weight", self.embed.weight, "vocab", None),
                 (p + "embed_positions.weight", self.pos, "replicate", None)]
        if self.norm is not None:
            specs += [(p + "final_layer_norm.weight", self.norm.weight, "replicate", None),
                      (p + "final_layer_norm.bias", self.norm.bias, "replicate", None)]
        if self.project_in is not None:
            specs += [(p + "project_in.weight", self.project_in.weight, "replicate", None),
                      (p + "project_out.weight", self.project_out.weight, "replicate", None)]
        if not cfg.tie_word_embeddings:
            specs.append(("lm_head.weight", self.lm_head.weight, "vocab", None))
        for i, layer in enumerate(self.layers):
            pre = f"{p}layers.{i}."
            a = layer.attn
            for nm, ln in (("self_attn_layer_norm", layer.self_attn_layer_norm),
                           ("final_layer_norm", layer.final_layer_norm)):
                specs += [(pre + nm + ".weight", ln.weight, "replicate", None),
                          (pre + nm + ".bias", ln.bias, "replicate", None)]
            rows = a.Hq * D
            for j, nm in enumerate(("q_proj", "k_proj", "v_proj")):
                specs.append((pre + f"self_attn.{nm}.weight", layer.qkv.weight, "fused", (j * rows, H, D)))
                if layer.qkv.bias is not None:
                    specs.append((pre + f"self_attn.{nm}.bias", layer.qkv.bias, "fused", (j * rows, H, D)))
            specs.append((pre + "self_attn.out_proj.weight", layer.out_proj.weight, "row", None))
            specs.append((pre + "fc1.weight", layer.mlp.fc1.weight, "col", None))
            specs.append((pre + "fc2.weight", layer.mlp.fc2.weight, "row", None))
            if layer.out_proj.bias is not None:
                specs += [(pre + "self_attn.out_proj.bias", layer.out_proj.bias, "replicate", None),
                          (pre + "fc1.bias", layer.mlp.fc1.bias, "col", None),
                          (pre + "fc2.bias", layer.mlp.fc2.bias, "replicate", None)]
        return specs

    @torch.no_grad()
    def forward(self, input_ids: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        x = self.embed(input_ids)
        if self.project_in is not None:
            x = self.project_in(x)
        x = x + F.embedding(meta.positions.long() + POS_OFFSET, self.pos)
        residual = None
        for layer in self.layers:
            x, residual = layer(x, residual, meta)
        if self.norm is not None:
            x, _ = self.norm(x, residual)
        elif residual is not None:
            x = x + residual
        return x

    @torch.no_grad()
    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        if self.project_out is not None:
            h = self.project_out(h)
        return self.lm_head(h)
