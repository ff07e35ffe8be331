"""Typed engine configuration with vLLM-compatible flag names.

Model architectures are described by ``ModelConfig`` (HF ``config.json``
field names). Presets cover the model families the reference's well-lit paths
deploy (SURVEY §2.3 shapes): Llama-3 8B/70B, Qwen3-32B, gpt-oss-20b/120b,
DeepSeek-V3/R1 (+ V2-Lite for scaled-down CI, reference
``.github/scripts/e2e/wide-ep-transform.sh:15-138``), OPT-125m-sized tiny
models for the CPU path, plus random tiny variants for tests.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Optional


@dataclass
class ModelConfig:
    model_type: str = "llama"
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: Optional[int] = None
    vocab_size: int = 128256
    max_position_embeddings: int = 131072
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    rms_norm_eps: float = 1e-5
    tie_word_embeddings: bool = False
    hidden_act: str = "silu"
    attention_bias: bool = False
    bos_token_id: int = 128000
    eos_token_id: Any = 128001
    # sliding window / sinks (gpt-oss): layer_types[i] in {"full_attention","sliding_attention"}
    sliding_window: int = 0
    layer_types: Optional[list] = None
    attention_sinks: bool = False
    # MoE (gpt-oss / DeepSeek / Mixtral)
    num_local_experts: int = 0
    num_experts_per_tok: int = 0
    moe_intermediate_size: int = 0
    n_shared_experts: int = 0
    first_k_dense_replace: int = 0
    router_aux_bias: bool = False
    swiglu_limit: float = 7.0
    # DeepSeek routing
    n_group: int = 1
    topk_group: int = 1
    routed_scaling_factor: float = 1.0
    norm_topk_prob: bool = False
    scoring_func: str = "softmax"
    # MLA (DeepSeek)
    q_lora_rank: Optional[int] = None
    kv_lora_rank: int = 0
    qk_nope_head_dim: int = 0
    qk_rope_head_dim: int = 0
    v_head_dim: int = 0
    # OPT (models/opt.py): token-embedding width when it differs from hidden_size
    # (project_in/out), pre- vs post-LayerNorm; attention_bias doubles as enable_bias
    word_embed_proj_dim: int = 0
    do_layer_norm_before: bool = True
    # multimodal (llava-style: vision tower + LM; models/vision.py)
    vision_config: Optional[dict] = None
    image_token_id: int = 0
    name: str = "custom"

    def __post_init__(self):
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads

    @property
    def is_moe(self) -> bool:
        return self.num_local_experts > 0

    @property
    def eos_ids(self) -> list[int]:
        e = self.eos_token_id
        return list(e) if isinstance(e, (list, tuple)) else [int(e)]

    def layer_window(self, i: int) -> int:
        if self.layer_types and self.layer_types[i] == "sliding_attention":
            return self.sliding_window
        return 0

    def num_params(self) -> int:
        d, L = self.hidden_size, self.num_hidden_layers
        hd = self.head_dim
        attn = d * (self.num_attention_heads + 2 * self.num_key_value_heads) * hd + self.num_attention_heads * hd * d
        if self.is_moe:
            mlp = self.num_local_experts * 3 * d * self.moe_intermediate_size + d * self.num_local_experts
        else:
            mlp = 3 * d * self.intermediate_size
        emb = self.vocab_size * d * (1 if self.tie_word_embeddings else 2)
        return L * (attn + mlp + 2 * d) + emb + d

    @classmethod
    def from_hf(cls, path_or_dict) -> "ModelConfig":
        if isinstance(path_or_dict, (str, os.PathLike)):
            p = os.path.join(path_or_dict, "config.json") if os.path.isdir(path_or_dict) else path_or_dict
            with open(p) as f:
                d = json.load(f)
        else:
            d = dict(path_or_dict)
        names = {f.name for f in dataclasses.fields(cls)}
        kw = {k: v for k, v in d.items() if k in names}
        if "num_experts" in d and "num_local_experts" not in d:
            kw["num_local_experts"] = d["num_experts"]
        if "n_routed_experts" in d:
            kw["num_local_experts"] = d["n_routed_experts"]
        if d.get("model_type") in ("deepseek_v3", "deepseek_v2"):
            kw["model_type"] = "deepseek"
        if d.get("model_type") == "opt":
            kw["intermediate_size"] = d.get("ffn_dim", 4 * d["hidden_size"])
            kw["num_key_value_heads"] = d["num_attention_heads"]
            kw["attention_bias"] = d.get("enable_bias", True)
            kw["hidden_act"] = d.get("activation_function", "relu")
            kw["tie_word_embeddings"] = d.get("tie_word_embeddings", True)
            kw.setdefault("rms_norm_eps", 1e-5)
        if d.get("model_type") == "gpt_oss":
            kw.setdefault("moe_intermediate_size", d.get("intermediate_size", 0))
            kw["attention_sinks"] = True
            kw["attention_bias"] = True
        return cls(**kw)


def _llama(name, d, ffn, L, hq, hkv, vocab=128256, **kw):
    base = dict(model_type="llama", hidden_size=d, intermediate_size=ffn, num_hidden_layers=L,
                num_attention_heads=hq, num_key_value_heads=hkv, vocab_size=vocab, name=name,
                rope_theta=500000.0,
                rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                              "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    base.update(kw)
    return ModelConfig(**base)


PRESETS: dict[str, ModelConfig] = {}


def _register(cfg: ModelConfig, *aliases):
    PRESETS[cfg.name] = cfg
    for a in aliases:
        PRESETS[a] = cfg


_register(_llama("llama-3-8b", 4096, 14336, 32, 32, 8), "meta-llama/Meta-Llama-3-8B",
          "meta-llama/Llama-3.1-8B-Instruct", "Llama-3-8B")
_register(_llama("llama-3-70b", 8192, 28672, 80, 64, 8), "meta-llama/Meta-Llama-3-70B",
          "meta-llama/Llama-3.3-70B-Instruct", "Llama-3-70B", "amd/Llama-3.3-70B-Instruct-FP8-KV")
_register(ModelConfig(model_type="qwen3", name="qwen3-32b", hidden_size=5120, intermediate_size=25600,
                      num_hidden_layers=64, num_attention_heads=64, num_key_value_heads=8, head_dim=128,
                      vocab_size=151936, rope_theta=1000000.0, rms_norm_eps=1e-6,
                      bos_token_id=151643, eos_token_id=151645), "Qwen/Qwen3-32B")
_register(ModelConfig(model_type="gpt_oss", name="gpt-oss-120b", hidden_size=2880, intermediate_size=2880,
                      moe_intermediate_size=2880, num_hidden_layers=36, num_attention_heads=64,
                      num_key_value_heads=8, head_dim=64, vocab_size=201088, rope_theta=150000.0,
                      rope_scaling={"rope_type": "yarn", "factor": 32.0, "beta_fast": 32.0, "beta_slow": 1.0,
                                    "original_max_position_embeddings": 4096},
                      num_local_experts=128, num_experts_per_tok=4, sliding_window=128,
                      layer_types=["sliding_attention", "full_attention"] * 18, attention_sinks=True,
                      attention_bias=True, bos_token_id=199998, eos_token_id=[200002, 199999]),
          "openai/gpt-oss-120b")
_register(ModelConfig(model_type="gpt_oss", name="gpt-oss-20b", hidden_size=2880, intermediate_size=2880,
                      moe_intermediate_size=2880, num_hidden_layers=24, num_attention_heads=64,
                      num_key_value_heads=8, head_dim=64, vocab_size=201088, rope_theta=150000.0,
                      rope_scaling={"rope_type": "yarn", "factor": 32.0, "beta_fast": 32.0, "beta_slow": 1.0,
                                    "original_max_position_embeddings": 4096},
                      num_local_experts=32, num_experts_per_tok=4, sliding_window=128,
                      layer_types=["sliding_attention", "full_attention"] * 12, attention_sinks=True,
                      attention_bias=True, bos_token_id=199998, eos_token_id=[200002, 199999]),
          "openai/gpt-oss-20b")
_DSV3_ROPE = {"rope_type": "yarn", "factor": 40.0, "beta_fast": 32.0, "beta_slow": 1.0, "mscale": 1.0,
              "mscale_all_dim": 1.0, "original_max_position_embeddings": 4096}
_register(ModelConfig(model_type="deepseek", name="deepseek-v3", hidden_size=7168, intermediate_size=18432,
                      moe_intermediate_size=2048, num_hidden_layers=61, num_attention_heads=128,
                      num_key_value_heads=128, vocab_size=129280, max_position_embeddings=163840,
                      rope_theta=10000.0, rope_scaling=_DSV3_ROPE, rms_norm_eps=1e-6, num_local_experts=256,
                      num_experts_per_tok=8, n_shared_experts=1, first_k_dense_replace=3, n_group=8, topk_group=4,
                      routed_scaling_factor=2.5, norm_topk_prob=True, scoring_func="sigmoid", router_aux_bias=True,
                      q_lora_rank=1536, kv_lora_rank=512, qk_nope_head_dim=128, qk_rope_head_dim=64,
                      v_head_dim=128, head_dim=192, bos_token_id=0, eos_token_id=1),
          "deepseek-ai/DeepSeek-V3", "deepseek-ai/DeepSeek-R1", "deepseek-ai/DeepSeek-R1-0528", "deepseek-r1")
_register(ModelConfig(model_type="deepseek", name="deepseek-v2-lite", hidden_size=2048, intermediate_size=10944,
                      moe_intermediate_size=1408, num_hidden_layers=27, num_attention_heads=16,
                      num_key_value_heads=16, vocab_size=102400, max_position_embeddings=163840,
                      rope_theta=10000.0, rope_scaling=dict(_DSV3_ROPE, mscale=0.707, mscale_all_dim=0.707),
                      rms_norm_eps=1e-6, num_local_experts=64, num_experts_per_tok=6, n_shared_experts=2,
                      first_k_dense_replace=1, q_lora_rank=None, kv_lora_rank=512, qk_nope_head_dim=128,
                      qk_rope_head_dim=64, v_head_dim=128, head_dim=192, bos_token_id=100000,
                      eos_token_id=100001), "deepseek-ai/DeepSeek-V2-Lite", "deepseek-ai/DeepSeek-V2-Lite-Chat")
_register(ModelConfig(model_type="mixtral", name="mixtral-8x7b", hidden_size=4096, intermediate_size=14336,
                      moe_intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
                      num_key_value_heads=8, head_dim=128, vocab_size=32000, rope_theta=1000000.0,
                      num_local_experts=8, num_experts_per_tok=2, norm_topk_prob=True, bos_token_id=1,
                      eos_token_id=2), "mistralai/Mixtral-8x7B-Instruct-v0.1")
_register(ModelConfig(model_type="qwen3_moe", name="qwen3-30b-a3b", hidden_size=2048, intermediate_size=6144,
                      moe_intermediate_size=768, num_hidden_layers=48, num_attention_heads=32,
                      num_key_value_heads=4, head_dim=128, vocab_size=151936, rope_theta=1000000.0,
                      rms_norm_eps=1e-6, num_local_experts=128, num_experts_per_tok=8, norm_topk_prob=True,
                      bos_token_id=151643, eos_token_id=151645), "Qwen/Qwen3-30B-A3B")
# further models the reference guides deploy (public HF configs)
_QW = dict(vocab_size=151936, rope_theta=1000000.0, rms_norm_eps=1e-6, bos_token_id=151643, eos_token_id=151645)
_register(ModelConfig(model_type="qwen3", name="qwen3-8b", hidden_size=4096, intermediate_size=12288,
                      num_hidden_layers=36, num_attention_heads=32, num_key_value_heads=8, head_dim=128, **_QW),
          "Qwen/Qwen3-8B")
_register(ModelConfig(model_type="qwen3", name="qwen3-0.6b", hidden_size=1024, intermediate_size=3072,
                      num_hidden_layers=28, num_attention_heads=16, num_key_value_heads=8, head_dim=128,
                      tie_word_embeddings=True, **_QW),
          "Qwen/Qwen3-0.6B", "Qwen/Qwen3-Embedding-0.6B")
_register(ModelConfig(model_type="qwen2", name="qwen2.5-3b", hidden_size=2048, intermediate_size=11008,
                      num_hidden_layers=36, num_attention_heads=16, num_key_value_heads=2, head_dim=128,
                      tie_word_embeddings=True, attention_bias=True, **dict(_QW, eos_token_id=151645)),
          "Qwen/Qwen2.5-3B-Instruct")
_register(_llama("llama-3.2-3b", 3072, 8192, 28, 24, 8, tie_word_embeddings=True,
                 rope_scaling={"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                               "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}),
          "meta-llama/Llama-3.2-3B-Instruct")
_register(ModelConfig(model_type="qwen3_moe", name="qwen3-coder-480b-a35b", hidden_size=6144, intermediate_size=8192,
                      moe_intermediate_size=2560, num_hidden_layers=62, num_attention_heads=96,
                      num_key_value_heads=8, head_dim=128, max_position_embeddings=262144,
                      num_local_experts=160, num_experts_per_tok=8, norm_topk_prob=True,
                      **dict(_QW, rope_theta=10000000.0)),
          "Qwen/Qwen3-Coder-480B-A35B-Instruct", "Qwen/Qwen3-Coder-480B-A35B-Instruct-FP8")
# multimodal (E/PD guide shape: Qwen2.5-VL-7B-class LM + ViT; image tokens = W*H/784)
_register(_llama("llama-3-8b-vl", 4096, 14336, 32, 32, 8, model_type="llava", image_token_id=128256,
                 vocab_size=128257, vision_config={"hidden_size": 1280, "num_layers": 32, "num_heads": 16}),
          "llava-llama-3-8b")
# OPT (the reference's CPU optimized-baseline model)
_register(ModelConfig(model_type="opt", name="opt-125m", hidden_size=768, intermediate_size=3072,
                      num_hidden_layers=12, num_attention_heads=12, num_key_value_heads=12, vocab_size=50272,
                      max_position_embeddings=2048, hidden_act="relu", attention_bias=True,
                      tie_word_embeddings=True, bos_token_id=2, eos_token_id=2), "facebook/opt-125m")
# tiny configs (CPU CI, smoke, GPU unit tests)
_register(ModelConfig(model_type="llama", name="tiny-llama", hidden_size=256, intermediate_size=512,
                      num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                      vocab_size=512, max_position_embeddings=4096, rope_theta=10000.0,
                      bos_token_id=1, eos_token_id=2))
_register(ModelConfig(model_type="llama", name="small-llama", hidden_size=1024, intermediate_size=2816,
                      num_hidden_layers=4, num_attention_heads=8, num_key_value_heads=2, head_dim=128,
                      vocab_size=32000, max_position_embeddings=8192, rope_theta=10000.0,
                      bos_token_id=1, eos_token_id=2), "opt-125m-sized")
_register(ModelConfig(model_type="opt", name="tiny-opt", hidden_size=256, intermediate_size=512,
                      num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=4, vocab_size=512,
                      max_position_embeddings=4096, hidden_act="relu", attention_bias=True,
                      tie_word_embeddings=True, bos_token_id=2, eos_token_id=2))
_register(ModelConfig(model_type="llava", name="tiny-vl", hidden_size=256, intermediate_size=512,
                      num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                      vocab_size=513, max_position_embeddings=4096, rope_theta=10000.0, bos_token_id=1,
                      eos_token_id=2, image_token_id=512,
                      vision_config={"hidden_size": 64, "num_layers": 2, "num_heads": 4,
                                     "max_pixels": 16 * 28 * 28, "min_pixels": 4 * 28 * 28}))
_register(ModelConfig(model_type="qwen3_moe", name="tiny-moe", hidden_size=256, intermediate_size=512,
                      moe_intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, head_dim=64, vocab_size=512, max_position_embeddings=4096,
                      rope_theta=10000.0, num_local_experts=8, num_experts_per_tok=2, norm_topk_prob=True,
                      bos_token_id=1, eos_token_id=2))
_register(ModelConfig(model_type="gpt_oss", name="tiny-gpt-oss", hidden_size=256, intermediate_size=256,
                      moe_intermediate_size=256, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, head_dim=64, vocab_size=512, rope_theta=10000.0,
                      num_local_experts=8, num_experts_per_tok=2, sliding_window=16,
                      layer_types=["sliding_attention", "full_attention"], attention_sinks=True,
                      attention_bias=True, bos_token_id=1, eos_token_id=2))


_register(ModelConfig(model_type="deepseek", name="tiny-deepseek", hidden_size=256, intermediate_size=512,
                      moe_intermediate_size=128, num_hidden_layers=3, num_attention_heads=20,
                      num_key_value_heads=20, vocab_size=512, max_position_embeddings=4096, rope_theta=10000.0,
                      rope_scaling=dict(_DSV3_ROPE, factor=4.0), rms_norm_eps=1e-6, num_local_experts=16,
                      num_experts_per_tok=4, n_shared_experts=1, first_k_dense_replace=1, n_group=4,
                      topk_group=2, routed_scaling_factor=2.5, norm_topk_prob=True, scoring_func="sigmoid",
                      router_aux_bias=True, q_lora_rank=96, kv_lora_rank=512, qk_nope_head_dim=128,
                      qk_rope_head_dim=64, v_head_dim=128, head_dim=192, bos_token_id=1, eos_token_id=2))


def get_model_config(name_or_path: str) -> ModelConfig:
    if name_or_path in PRESETS:
        return dataclasses.replace(PRESETS[name_or_path])
    if os.path.exists(name_or_path):
        return ModelConfig.from_hf(name_or_path)
    raise ValueError(f"unknown model {name_or_path!r}; presets: {sorted(set(c.name for c in PRESETS.values()))}")


@dataclass
class CacheConfig:
    block_size: int = 64
    gpu_memory_utilization: float = 0.92
    kv_cache_memory_bytes: Optional[int] = None
    num_gpu_blocks: Optional[int] = None
    enable_prefix_caching: bool = True
    kv_cache_dtype: str = "auto"
    # decode attention reads a prefix shared by several running sequences once
    # per group (ops.shared_prefix_plan; needs prefix caching to share blocks)
    shared_prefix_decode: bool = True
    # hybrid KV-cache manager (engine/hybrid_kv.py): None = on for models with sliding-window
    # layers unless a KV connector needs whole-model blocks; False = off
    # (--disable-hybrid-kv-cache-manager); True = requested (--no-disable-hybrid-kv-cache-manager)
    hybrid_kv_cache_manager: Optional[bool] = None

    def __post_init__(self):
        # the attention kernels index blocks with shifts/masks
        if self.block_size <= 0 or self.block_size & (self.block_size - 1):
            raise ValueError(f"block_size must be a power of two, got {self.block_size}")


@dataclass
class SchedulerConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: int = 32768
    enable_chunked_prefill: bool = True
    # step N+1 is scheduled and launched before step N's sampled tokens reach the host (its decode
    # inputs are gathered on the device); the host turns step N into outputs while N+1 runs.
    # Applies to single-rank engines (TP / DP-lockstep / P/D-connector engines step synchronously).
    async_scheduling: bool = True
    policy: str = "fcfs"  # or "priority"
    long_prefill_token_threshold: int = 0
    # Steps carrying a prefill chunk are trimmed so their token count (the M of
    # every dense GEMM) is a multiple of this: hipBLASLt's tile/stream-K choice
    # is erratic at arbitrary M (Llama-3-70B layer at M=5064 costs more than at
    # M=6000, profiles/gemm_prefill_odd_m.txt) and the committed TunableOp table
    # covers the aligned sizes. -1 = auto (512 on GPU, off on CPU), 0 = off.
    prefill_token_align: int = -1


@dataclass
class ParallelConfig:
    tensor_parallel_size: int = 1
    data_parallel_size: int = 1
    data_parallel_rank: int = 0
    enable_expert_parallel: bool = False
    distributed_backend: str = "nccl"
    all2all_backend: str = "allgather_reducescatter"  # wide-EP token exchange (parallel/ep.py)
    disable_custom_all_reduce: bool = False  # TP all-reduce over the symm IPC heap (parallel/symm.py)
    enable_eplb: bool = False  # expert load balancing with redundant experts (parallel/eplb.py)
    eplb_config: Optional[dict] = None  # {"window_size", "step_interval", "num_redundant_experts"}
    enable_dbo: bool = False  # dual-batch overlap of EP exchange with compute (decode steps)
    dbo_decode_token_threshold: int = 32
    dbo_prefill_token_threshold: int = 32  # steps with prefills (reference prefill.yaml:83-84)


@dataclass
class EngineConfig:
    model: str = "tiny-llama"
    model_config: ModelConfig = field(default_factory=ModelConfig)
    cache: CacheConfig = field(default_factory=CacheConfig)
    sched: SchedulerConfig = field(default_factory=SchedulerConfig)
    parallel: ParallelConfig = field(default_factory=ParallelConfig)
    device: str = "cuda"
    dtype: str = "bfloat16"
    seed: int = 0
    load_format: str = "dummy"  # "dummy" (random init) | "safetensors"
    weights_path: Optional[str] = None
    quantization: Optional[str] = None  # None | "fp8" (W8A8: per-channel fp8 weights, per-token activations)
    # | "mxfp4" (routed experts in MXFP4, e2m1 + E8M0 per 32; other linears as fp8)
    tokenizer: Optional[str] = None
    served_model_name: Optional[str] = None
    enforce_eager: bool = False
    cuda_graph_max_bs: int = 256
    kv_transfer_config: Optional[dict] = None
    kv_events_config: Optional[dict] = None
    kv_offload_config: Optional[dict] = None
    max_loras: int = 0
    enable_lora: bool = False
    max_lora_rank: int = 16
    lora_modules: Optional[dict] = None  # name -> adapter dir, loaded at start-up

    @property
    def served_name(self) -> str:
        return self.served_model_name or self.model

    @classmethod
    def create(cls, model: str = "tiny-llama", **kw) -> "EngineConfig":
        mc = kw.pop("model_config", None) or get_model_config(model)
        sub = {"cache": CacheConfig, "sched": SchedulerConfig, "parallel": ParallelConfig}
        parts = {k: c() for k, c in sub.items()}
        top = {}
        for k, v in kw.items():
            placed = False
            for name, c in sub.items():
                if k in {f.name for f in dataclasses.fields(c)}:
                    setattr(parts[name], k, v)
                    placed = True
            if not placed:
                top[k] = v
        cfg = cls(model=model, model_config=mc, **parts, **top)
        cfg.sched.max_model_len = min(cfg.sched.max_model_len, mc.max_position_embeddings)
        if cfg.sched.prefill_token_align < 0:
            cfg.sched.prefill_token_align = (int(os.environ.get("LLMD_PREFILL_ALIGN", "512"))
                                             if str(cfg.device).startswith("cuda") else 0)
        return cfg


def _json_arg(s):
    return json.loads(s) if s else None


def add_engine_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    """vLLM-compatible engine flags (subset with identical semantics)."""
    p.add_argument("--model", default="tiny-llama")
    p.add_argument("--served-model-name", default=None)
    p.add_argument("--tokenizer", default=None)
    p.add_argument("--load-format", default="dummy", choices=["dummy", "safetensors", "auto"])
    p.add_argument("--weights-path", default=None)
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--device", default="cuda")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--block-size", type=int, default=64)
    p.add_argument("--quantization", "-q", default=None, choices=[None, "fp8", "mxfp4"],
                   help="fp8: online W8A8 quantisation of the dense linears (hipBLASLt fp8 GEMM); "
                   "mxfp4: routed experts in MXFP4 (gpt-oss's format), dense linears as fp8")
    p.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "bfloat16", "fp8", "fp8_e4m3"],
                   help="KV cache storage: bf16 (auto) or OCP fp8 e4m3fn")
    p.add_argument("--gpu-memory-utilization", type=float, default=0.92)
    p.add_argument("--kv-cache-memory-bytes", type=int, default=None)
    p.add_argument("--num-gpu-blocks-override", type=int, default=None)
    p.add_argument("--no-enable-prefix-caching", action="store_true")
    p.add_argument("--disable-shared-prefix-decode", action="store_true",
                   help="read shared cached prefixes per sequence in decode attention (no cascade kernel)")
    p.add_argument("--max-num-seqs", type=int, default=256)
    p.add_argument("--max-num-batched-tokens", type=int, default=8192)
    p.add_argument("--max-model-len", type=int, default=32768)
    p.add_argument("--tensor-parallel-size", "-tp", type=int, default=1)
    p.add_argument("--data-parallel-size", "-dp", type=int, default=1)
    p.add_argument("--data-parallel-rank", type=int, default=0)
    p.add_argument("--enable-expert-parallel", action="store_true")
    p.add_argument("--all2all-backend", default="allgather_reducescatter",
                   choices=["allgather_reducescatter", "alltoall", "symm_ll", "symm_ht", "deepep_low_latency",
                            "deepep_high_throughput"])
    p.add_argument("--disable-custom-all-reduce", action="store_true")
    p.add_argument("--enable-eplb", action="store_true")
    p.add_argument("--eplb-config", type=_json_arg, default=None)
    p.add_argument("--enable-dbo", action="store_true")
    p.add_argument("--dbo-decode-token-threshold", type=int, default=32)
    p.add_argument("--dbo-prefill-token-threshold", type=int, default=32)
    p.add_argument("--enforce-eager", action="store_true")
    p.add_argument("--kv-transfer-config", type=_json_arg, default=None)
    p.add_argument("--kv-events-config", type=_json_arg, default=None)
    p.add_argument("--kv-offload-config", type=_json_arg, default=None)
    p.add_argument("--scheduling-policy", default="fcfs", choices=["fcfs", "priority"])
    p.add_argument("--prefill-token-align", type=int, default=-1,
                   help="trim prefill-carrying steps to a multiple of this many tokens (GEMM M); "
                        "-1 auto (512 on GPU), 0 off")
    p.add_argument("--enable-lora", action="store_true")
    p.add_argument("--max-loras", type=int, default=4)
    p.add_argument("--max-lora-rank", type=int, default=16)
    p.add_argument("--lora-modules", nargs="*", default=None, help="name=path adapters loaded at start-up")
    # vLLM flags the reference's guides pass, mapped onto this engine
    p.add_argument("--hf-overrides", type=_json_arg, default=None,
                   help="JSON of model-config fields to override (HF names, e.g. num_hidden_layers)")
    p.add_argument("--disable-sliding-window", action="store_true",
                   help="full attention on every layer (sliding-window layers included)")
    p.add_argument("--max-cudagraph-capture-size", type=int, default=None,
                   help="largest decode batch captured as a hipGraph")
    p.add_argument("--compilation-config", "-O", type=_json_arg, default=None,
                   help="vLLM compilation config: cudagraph_capture_sizes / max_cudagraph_capture_size set the "
                        "hipGraph buckets, cudagraph_mode NONE = --enforce-eager; other keys are ignored "
                        "(no tracing compiler: the hot ops are HIP kernels)")
    # accepted for command-line compatibility; no effect on this engine
    for f in ("--trust-remote-code", "--enable-cumem-allocator", "--enable-ep-weight-filter",
              "--enable-prefiller-sampling",
              "--data-parallel-hybrid-lb", "--data-parallel-multi-port-external-lb"):
        p.add_argument(f, action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--async-scheduling", dest="async_scheduling", action="store_true", default=True,
                   help="launch step N+1 before step N's tokens reach the host (default on)")
    p.add_argument("--no-async-scheduling", dest="async_scheduling", action="store_false")
    p.add_argument("--disable-hybrid-kv-cache-manager", action="store_true",
                   help="every layer keeps full-length KV (no separate sliding-window pool)")
    p.add_argument("--no-disable-hybrid-kv-cache-manager", action="store_true",
                   help="request the hybrid KV-cache manager (sliding-window layers in their own pool)")
    for f in ("--tokenizer-mode", "--attention-backend", "--moe-backend", "--data-parallel-address",
              "--data-parallel-rpc-port", "--data-parallel-supervisor-port"):
        p.add_argument(f, default=None, help=argparse.SUPPRESS)
    p.add_argument("--data-parallel-size-local", type=int, default=None,
                   help="DP ranks on this node (must equal the local torchrun ranks / tp)")
    p.add_argument("--data-parallel-start-rank", type=int, default=0,
                   help="global DP rank of this node's first rank (multi-node DP)")
    return p


def _model_config_from_args(a) -> Optional["ModelConfig"]:
    ov = dict(getattr(a, "hf_overrides", None) or {})
    if not ov and not getattr(a, "disable_sliding_window", False):
        return None
    mc = get_model_config(a.model)
    unknown = [k for k in ov if not hasattr(mc, k)]
    if unknown:
        raise ValueError(f"--hf-overrides: unknown model-config fields {unknown}")
    mc = dataclasses.replace(mc, **ov)
    if getattr(a, "disable_sliding_window", False):
        mc = dataclasses.replace(mc, sliding_window=0,
                                 layer_types=["full_attention"] * mc.num_hidden_layers if mc.layer_types else
                                 mc.layer_types)
    return mc


def _graph_max_bs(a) -> tuple[Optional[int], bool]:
    """(largest captured decode batch, eager) from the vLLM graph flags."""
    cc = getattr(a, "compilation_config", None) or {}
    eager = a.enforce_eager or str(cc.get("cudagraph_mode", "")).upper() == "NONE"
    bs = getattr(a, "max_cudagraph_capture_size", None) or cc.get("max_cudagraph_capture_size")
    if bs is None and cc.get("cudagraph_capture_sizes"):
        bs = max(int(x) for x in cc["cudagraph_capture_sizes"])
    return (int(bs) if bs else None), eager


def engine_config_from_args(a) -> EngineConfig:
    graph_bs, eager = _graph_max_bs(a)
    extra = {}
    mc = _model_config_from_args(a)
    if mc is not None:
        extra["model_config"] = mc
    if graph_bs is not None:
        extra["cuda_graph_max_bs"] = graph_bs
    return EngineConfig.create(
        a.model, **extra, served_model_name=a.served_model_name, tokenizer=a.tokenizer,
        load_format=a.load_format, weights_path=a.weights_path, dtype=a.dtype, device=a.device,
        seed=a.seed, block_size=a.block_size, kv_cache_dtype=getattr(a, "kv_cache_dtype", "auto"),
        quantization=getattr(a, "quantization", None), gpu_memory_utilization=a.gpu_memory_utilization,
        kv_cache_memory_bytes=a.kv_cache_memory_bytes, num_gpu_blocks=a.num_gpu_blocks_override,
        enable_prefix_caching=not a.no_enable_prefix_caching, max_num_seqs=a.max_num_seqs,
        shared_prefix_decode=not getattr(a, "disable_shared_prefix_decode", False),
        hybrid_kv_cache_manager=(False if getattr(a, "disable_hybrid_kv_cache_manager", False) else
                                 True if getattr(a, "no_disable_hybrid_kv_cache_manager", False) else None),
        max_num_batched_tokens=a.max_num_batched_tokens, max_model_len=a.max_model_len,
        tensor_parallel_size=a.tensor_parallel_size, data_parallel_size=a.data_parallel_size,
        data_parallel_rank=a.data_parallel_rank, enable_expert_parallel=a.enable_expert_parallel,
        all2all_backend=getattr(a, "all2all_backend", "allgather_reducescatter"),
        disable_custom_all_reduce=getattr(a, "disable_custom_all_reduce", False),
        enable_eplb=getattr(a, "enable_eplb", False), eplb_config=getattr(a, "eplb_config", None),
        enable_dbo=getattr(a, "enable_dbo", False),
        dbo_decode_token_threshold=getattr(a, "dbo_decode_token_threshold", 32),
        dbo_prefill_token_threshold=getattr(a, "dbo_prefill_token_threshold", 32),
        enforce_eager=eager, kv_transfer_config=a.kv_transfer_config,
        kv_events_config=a.kv_events_config, kv_offload_config=a.kv_offload_config,
        policy=a.scheduling_policy, prefill_token_align=getattr(a, "prefill_token_align", -1),
        async_scheduling=getattr(a, "async_scheduling", True),
        enable_lora=getattr(a, "enable_lora", False),
        max_loras=getattr(a, "max_loras", 4), max_lora_rank=getattr(a, "max_lora_rank", 16),
        lora_modules=dict(m.split("=", 1) for m in (getattr(a, "lora_modules", None) or [])) or None)
