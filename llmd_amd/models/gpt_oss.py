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
With expert parallelism every rank owns E/EP experts: under TP the tokens are
replicated and one all-reduce sums the expert owners' contributions; under
DP attention (wide-EP) tokens are exchanged with ``parallel/ep.py``
(all-gather/reduce-scatter or all-to-all dispatch/combine).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from llmd_amd import ops
from llmd_amd.engine.config import ModelConfig
from llmd_amd.parallel.comm import tp_all_reduce
from llmd_amd.parallel import eplb
from llmd_amd.parallel.ep import ep_active, moe_ep
from llmd_amd.parallel.state import get_state

from .layers import _init_weight, run_experts
from .llama import LlamaDecoderLayer, LlamaForCausalLM


class GptOssMoE(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, device, ep: bool = False):
        super().__init__()
        st = get_state()
        self.ep = ep and st.ep_size > 1
        self.dp_ep = self.ep and ep_active()   # DP attention: exchange tokens with expert owners
        self.tp = st.tp_size
        self.ep_size = st.ep_size if self.ep else 1
        self.ep_rank = st.ep_rank if self.ep else 0
        E = cfg.num_local_experts
        assert E % self.ep_size == 0
        self.E, self.E_local = E, E // self.ep_size
        self.k = cfg.num_experts_per_tok
        self.eplb = None
        if self.dp_ep and eplb.config().enabled:  # physical slots incl. redundant replicas
            self.eplb = eplb.EplbLayer(E, self.ep_size, self.ep_rank, device, eplb.config().num_redundant_experts)
            self.E_local = self.eplb.P_local
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
            return run_experts(self, x, ids, w, ops.ACT_SWIGLU_OAI, self.alpha, self.limit, b1=self.b1, b2=self.b2)
        fn = lambda xx, ii, ww: run_experts(self, xx, ii, ww, ops.ACT_SWIGLU_OAI,  # noqa: E731
                                            self.alpha, self.limit, b1=self.b1, b2=self.b2)
        if self.dp_ep:  # DP+EP: all-gather/reduce-scatter or all-to-all dispatch/combine
            if self.eplb is not None:
                ids = self.eplb.route(ids)
            return moe_ep(x, ids, w, self.E_local, fn)
        # EP over TP ranks (tokens replicated): local experts only, then one all-reduce.
        # b2 is added once per (token, expert) by the owner rank, so the sum stays exact.
        lo = self.ep_rank * self.E_local
        local = (ids >= lo) & (ids < lo + self.E_local)
        y = fn(x, torch.where(local, ids - lo, torch.full_like(ids, -1)), torch.where(local, w, torch.zeros_like(w)))
        return tp_all_reduce(y)


    def expert_params(self) -> list:
        ps = [self.w1.data, self.b1.data, self.w2.data, self.b2.data]
        for nm in ("w1_scale", "w2_scale"):
            if hasattr(self, nm):
                ps.append(getattr(self, nm).data)
        return ps


class GptOssDecoderLayer(LlamaDecoderLayer):
    def _make_mlp(self, cfg, idx, device):
        return GptOssMoE(cfg, device, ep=True)


class GptOssForCausalLM(LlamaForCausalLM):
    layer_cls = GptOssDecoderLayer

    def _mlp_specs(self, pre: str, mlp) -> list:
        """HF gpt-oss MoE tensors: router.{weight,bias}, experts.gate_up_proj [E, d, 2F]
        (gate/up interleaved columns), experts.down_proj [E, F, d] (+ biases)."""
        if mlp.eplb is not None:  # physical slots -> logical experts (replicas load their expert)
            sel = list(mlp.eplb.local_logical())
        else:
            lo, n = mlp.ep_rank * mlp.E_local, mlp.E_local
            sel = (lo, n)
        return [(pre + "mlp.router.weight", mlp.router_w, "replicate", None),
                (pre + "mlp.router.bias", mlp.router_b, "replicate", None),
                (pre + "mlp.experts.gate_up_proj", mlp.w1, "experts_t", sel),
                (pre + "mlp.experts.gate_up_proj_bias", mlp.b1, "experts", sel),
                (pre + "mlp.experts.down_proj", mlp.w2, "experts_t", sel),
                (pre + "mlp.experts.down_proj_bias", mlp.b2, "experts", sel)]
