"""Mixtral / Qwen3-MoE: Llama-architecture attention (Qwen3: per-head q/k
RMSNorm) with a routed-expert MLP - softmax router over all experts, top-k
with renormalisation, SiLU-gated experts, no shared expert.

The MoE path is the same native one as gpt-oss / DeepSeek (moe_topk ->
moe_align -> two grouped MFMA GEMMs with the SiLU gate fused into GEMM 1 ->
deterministic combine; block-fp8 experts under ``--quantization fp8``),
expert-parallel over TP ranks (one all-reduce) or over DP ranks (wide-EP
token exchange, EPLB). HF expert tensors (``mlp.experts.{e}.gate_proj`` /
``up_proj`` / ``down_proj`` for Qwen3-MoE, ``block_sparse_moe.experts.{e}.w1``
/ ``w3`` / ``w2`` for Mixtral) are interleaved into the [E, 2F, d] layout on load.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from llmd_amd import ops
from llmd_amd.engine.config import ModelConfig
from llmd_amd.parallel import eplb
from llmd_amd.parallel.comm import tp_all_reduce
from llmd_amd.parallel.ep import ep_active, moe_ep
from llmd_amd.parallel.state import get_state

from .layers import _init_weight, run_experts
from .llama import LlamaDecoderLayer, LlamaForCausalLM


class SparseMoE(torch.nn.Module):
    def __init__(self, cfg: ModelConfig, device):
        super().__init__()
        st = get_state()
        self.dp_ep = ep_active()
        self.n_ep = st.ep_size if self.dp_ep else st.tp_size
        self.r_ep = st.ep_rank if self.dp_ep else st.tp_rank
        self.tp = st.tp_size
        E, d = cfg.num_local_experts, cfg.hidden_size
        Fh = cfg.moe_intermediate_size or cfg.intermediate_size
        if E % self.n_ep:
            raise ValueError(f"{E} experts do not split over EP={self.n_ep}")
        self.E, self.E_local, self.k = E, E // self.n_ep, cfg.num_experts_per_tok
        self.lo = self.r_ep * self.E_local
        self.renorm = cfg.norm_topk_prob
        self.eplb = None
        if self.dp_ep and eplb.config().enabled:
            self.eplb = eplb.EplbLayer(E, self.n_ep, self.r_ep, device, eplb.config().num_redundant_experts)
            self.E_local = self.eplb.P_local
        dt = torch.bfloat16
        self.gate = torch.nn.Parameter(_init_weight(torch.empty(E, d, device=device, dtype=dt), 0.02),
                                       requires_grad=False)
        self.w1 = torch.nn.Parameter(_init_weight(torch.empty(self.E_local, 2 * Fh, d, device=device, dtype=dt),
                                                  0.02), requires_grad=False)
        self.w2 = torch.nn.Parameter(_init_weight(torch.empty(self.E_local, d, Fh, device=device, dtype=dt),
                                                  0.02), requires_grad=False)

    def forward(self, x):
        logits = F.linear(x, self.gate).float()
        ids, w = ops.moe_topk(logits, self.k, scoring=0, renorm=self.renorm)
        fn = lambda xx, ii, ww: run_experts(self, xx, ii, ww, ops.ACT_SILU)  # noqa: E731
        if self.dp_ep:
            if self.eplb is not None:
                ids = self.eplb.route(ids)
            return moe_ep(x, ids, w, self.E_local, fn)
        if self.n_ep > 1:  # experts over TP ranks, tokens replicated: local experts + one all-reduce
            local = (ids >= self.lo) & (ids < self.lo + self.E_local)
            ids = torch.where(local, ids - self.lo, torch.full_like(ids, -1))
            w = torch.where(local, w, torch.zeros_like(w))
        y = fn(x, ids, w)
        return tp_all_reduce(y) if self.tp > 1 else y

    def expert_params(self) -> list:
        ps = [self.w1.data, self.w2.data]
        for nm in ("w1_scale", "w2_scale"):
            if hasattr(self, nm):
                ps.append(getattr(self, nm).data)
        return ps


class MoELlamaDecoderLayer(LlamaDecoderLayer):
    def _make_mlp(self, cfg, idx, device):
        return SparseMoE(cfg, device)


class MoELlamaForCausalLM(LlamaForCausalLM):
    layer_cls = MoELlamaDecoderLayer

    def _mlp_specs(self, pre: str, mlp) -> list:
        if mlp.eplb is not None:
            logical = mlp.eplb.local_logical()
        else:
            logical = [mlp.lo + i for i in range(mlp.E_local)]
        mixtral = self.cfg.model_type == "mixtral"
        gate_name = pre + ("block_sparse_moe.gate.weight" if mixtral else "mlp.gate.weight")
        specs = [(gate_name, mlp.gate, "replicate", None)]
        for el, e in enumerate(logical):
            if mixtral:
                ep = f"{pre}block_sparse_moe.experts.{e}."
                names = (ep + "w1.weight", ep + "w3.weight", ep + "w2.weight")
            else:
                ep = f"{pre}mlp.experts.{e}."
                names = (ep + "gate_proj.weight", ep + "up_proj.weight", ep + "down_proj.weight")
            specs += [(names[0], mlp.w1[el], "rows", (0, 2)), (names[1], mlp.w1[el], "rows", (1, 2)),
                      (names[2], mlp.w2[el], "replicate", None)]
        return specs
