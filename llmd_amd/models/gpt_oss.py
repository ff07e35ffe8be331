"""gpt-oss (20b / 120b) on the paged-KV engine: the model the reference's P/D
and tiered-prefix-cache guides serve (guides/pd-disaggregation/README.md:7-13,
guides/tiered-prefix-cache/benchmark-results-gpt-oss-120b.md).

Architecture: GQA attention (64 Q / 8 KV heads, head_dim 64) with q/k/v/o
biases and learned per-head attention sinks, alternating sliding-window (128)
and full attention layers, YaRN RoPE; MoE MLP with 32/128 experts, top-4,
softmax over the selected router logits, clamped SwiGLU (alpha 1.702,
limit 7) with expert biases.

MoE execution: native gating (``moe_topk``), expert alignment and two MFMA
grouped GEMMs with fused activation / bias, deterministic weighted combine
(``llmd_amd/csrc/ops/moe.hip``). Expert weights use the interleaved
gate/up row layout ([E, 2F, d]) so the activation fuses into GEMM-1.
With expert parallelism (EP = world) every rank owns E/EP experts; tokens
are all-gathered, each rank computes its experts' contributions, and a
reduce-scatter returns the token rows (the reference's
``allgather_reducescatter`` all2all backend).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from llmd_amd import ops
from llmd_amd.engine.config import ModelConfig
from llmd_amd.parallel.comm import ep_all_gather, ep_reduce_scatter
from llmd_amd.parallel.state import get_state

from .layers import _init_weight
from .llama import LlamaDecoderLayer, LlamaForCausalLM


class GptOssMoE(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, device, ep: bool = False):
        super().__init__()
        st = get_state()
        self.ep = ep and st.ep_size > 1
        self.ep_size = st.ep_size if self.ep else 1
        self.ep_rank = st.ep_rank if self.ep else 0
        E = cfg.num_local_experts
        assert E % self.ep_size == 0
        self.E, self.E_local = E, E // self.ep_size
        self.k = cfg.num_experts_per_tok
        d, Fh = cfg.hidden_size, cfg.moe_intermediate_size
        dt = torch.bfloat16
        self.router_w = torch.nn.Parameter(_init_weight(torch.empty(E, d, device=device, dtype=dt), 0.02),
                                           requires_grad=False)
        self.router_b = torch.nn.Parameter(torch.zeros(E, device=device, dtype=dt), requires_grad=False)
        self.w1 = torch.nn.Parameter(_init_weight(torch.empty(self.E_local, 2 * Fh, d, device=device, dtype=dt), 0.02),
                                     requires_grad=False)
        self.b1 = torch.nn.Parameter(torch.zeros(self.E_local, 2 * Fh, device=device, dtype=dt), requires_grad=False)
        self.w2 = torch.nn.Parameter(_init_weight(torch.empty(self.E_local, d, Fh, device=device, dtype=dt), 0.02),
                                     requires_grad=False)
        self.b2 = torch.nn.Parameter(torch.zeros(self.E_local, d, device=device, dtype=dt), requires_grad=False)
        self.alpha, self.limit = 1.702, cfg.swiglu_limit

    def forward(self, x):
        T = x.shape[0]
        logits = F.linear(x, self.router_w, self.router_b).float()
        ids, w = ops.moe_topk(logits, self.k, scoring=2)
        if not self.ep:
            return ops.moe_experts(x, ids, w, self.w1, self.w2, ops.ACT_SWIGLU_OAI, self.alpha, self.limit,
                                   b1=self.b1, b2=self.b2)
        # EP: all-gather tokens + routing, compute local experts, reduce-scatter
        xs = ep_all_gather(x)
        ids_all = ep_all_gather(ids)
        w_all = ep_all_gather(w)
        lo = self.ep_rank * self.E_local
        local = (ids_all >= lo) & (ids_all < lo + self.E_local)
        lids = torch.where(local, ids_all - lo, torch.full_like(ids_all, -1))
        lw = torch.where(local, w_all, torch.zeros_like(w_all))
        y = ops.moe_experts(xs, lids, lw, self.w1, self.w2, ops.ACT_SWIGLU_OAI, self.alpha, self.limit,
                            b1=self.b1, b2=self.b2)
        return ep_reduce_scatter(y)


class GptOssDecoderLayer(LlamaDecoderLayer):
    def _make_mlp(self, cfg, idx, device):
        return GptOssMoE(cfg, device, ep=True)


class GptOssForCausalLM(LlamaForCausalLM):
    layer_cls = GptOssDecoderLayer
