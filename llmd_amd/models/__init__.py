"""Model registry: HF ``model_type`` -> implementation."""
from __future__ import annotations

from llmd_amd.engine.config import ModelConfig


def model_class(cfg: ModelConfig):
    t = cfg.model_type
    if t in ("llama", "qwen3", "qwen2", "mistral"):
        from .llama import LlamaForCausalLM

        return LlamaForCausalLM
    if t == "opt":
        from .opt import OPTForCausalLM

        return OPTForCausalLM
    if t == "llava":
        from .vision import LlavaForCausalLM

        return LlavaForCausalLM
    if t == "gpt_oss":
        from .gpt_oss import GptOssForCausalLM

        return GptOssForCausalLM
    if t in ("deepseek", "deepseek_v3", "deepseek_v2"):
        from .deepseek import DeepseekForCausalLM

        return DeepseekForCausalLM
    if t in ("mixtral", "qwen3_moe"):
        from .moe_llama import MoELlamaForCausalLM

        return MoELlamaForCausalLM
    raise ValueError(f"unsupported model_type {t!r}")


def build_model(cfg: ModelConfig, device="cuda", max_pos: int = 32768):
    return model_class(cfg)(cfg, device=device, max_pos=max_pos)
