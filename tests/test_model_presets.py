"""Model presets for the models the reference guides deploy resolve to a
supported architecture with consistent shapes, and the architecture features
they rely on (Qwen2 q/k/v bias, tied embeddings, Qwen3 q/k norm) run through
the engine and round-trip an HF-format checkpoint on CPU."""
import dataclasses

import numpy as np
import pytest
import torch

from llmd_amd.engine.config import EngineConfig, get_model_config
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams
from llmd_amd.models import model_class

GUIDE_MODELS = ["Qwen/Qwen3-32B", "Qwen/Qwen3-8B", "Qwen/Qwen3-0.6B", "Qwen/Qwen3-Embedding-0.6B",
                "openai/gpt-oss-120b", "deepseek-ai/DeepSeek-R1-0528", "meta-llama/Llama-3.2-3B-Instruct",
                "meta-llama/Llama-3.1-8B-Instruct", "Qwen/Qwen2.5-3B-Instruct", "amd/Llama-3.3-70B-Instruct-FP8-KV",
                "Qwen/Qwen3-Coder-480B-A35B-Instruct-FP8"]


@pytest.mark.parametrize("name", GUIDE_MODELS)
def test_guide_model_presets_resolve(name):
    c = get_model_config(name)
    assert model_class(c) is not None
    assert c.num_attention_heads % c.num_key_value_heads == 0
    if c.model_type != "deepseek":
        assert c.head_dim * c.num_attention_heads >= c.hidden_size // 2


@pytest.mark.parametrize("base,kw", [
    ("Qwen/Qwen2.5-3B-Instruct", {}),              # qkv bias + tied embeddings
    ("Qwen/Qwen3-0.6B", {}),                       # q/k norm + tied embeddings
    ("meta-llama/Llama-3.2-3B-Instruct", {}),      # llama3 rope scaling + tied embeddings
])
def test_architecture_features_run_and_roundtrip(tmp_path, base, kw):
    from llmd_amd.engine import config as C
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    mc = dataclasses.replace(get_model_config(base), name=f"mini-{base}", hidden_size=256, intermediate_size=512,
                             num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                             vocab_size=512, **kw)
    C._register(mc)
    path = str(tmp_path / "m.safetensors")
    m = build_model(mc, device="cpu", max_pos=600)
    if mc.attention_bias:
        for layer in m.layers:
            torch.nn.init.normal_(layer.qkv.bias, std=2.0)  # non-zero: the bias must be loaded and used
    save_safetensors(export_hf(m), path)
    path0 = None
    if mc.attention_bias:
        for layer in m.layers:
            layer.qkv.bias.data.zero_()
        path0 = str(tmp_path / "m0.safetensors")
        save_safetensors(export_hf(m), path0)

    def eng(weights):
        return LLMEngine(EngineConfig.create(mc.name, device="cpu", block_size=16, num_gpu_blocks=64,
                                             max_num_batched_tokens=64, max_num_seqs=4, max_model_len=256,
                                             enforce_eager=True, load_format="safetensors", weights_path=weights))

    prompts = [np.random.default_rng(1).integers(3, 500, size=30).tolist()]
    sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    a = eng(path).generate(prompts, sp)[0].output_token_ids
    b = eng(path).generate(prompts, sp)[0].output_token_ids
    assert a == b and len(a) == 4  # the checkpoint fully determines the outputs (no random leftovers)
    if path0 is not None:
        e0 = eng(path0)
        lp = lambda e: e.generate(prompts, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True,  # noqa: E731
                                                          logprobs=1))[0].output_logprobs[0]
        assert abs(lp(eng(path)) - lp(e0)) > 1e-4  # q/k/v bias loaded and applied
