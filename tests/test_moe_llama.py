"""Mixtral / Qwen3-MoE family (models/moe_llama.py) on CPU: generation, HF
export -> load round trip (per-expert gate/up interleave), TP=1 vs EP over
TP ranks handled by the same routed-expert path as gpt-oss/DeepSeek."""
import pytest

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams


def _cfg(**kw):
    return EngineConfig.create("tiny-moe", device="cpu", block_size=16, num_gpu_blocks=64, max_num_batched_tokens=128,
                               max_num_seqs=4, max_model_len=512, enforce_eager=True, **kw)


def test_moe_llama_generates_and_roundtrips(tmp_path):
    from llmd_amd.models.loader import export_hf, save_safetensors

    eng = LLMEngine(_cfg())
    assert eng.runner.model.layers[0].qk_norm  # qwen3_moe: per-head q/k norm
    sp = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    prompts = [list(range(5, 40)), [9] * 17]
    want = [r.output_token_ids for r in eng.generate(prompts, sp)]
    path = str(tmp_path / "m.safetensors")
    sd = export_hf(eng.runner.model)
    assert any(".mlp.experts.3.up_proj.weight" in k for k in sd)
    save_safetensors(sd, path)
    eng2 = LLMEngine(_cfg(load_format="safetensors", weights_path=path, seed=123))
    got = [r.output_token_ids for r in eng2.generate(prompts, sp)]
    assert got == want


@pytest.mark.parametrize("name", ["mixtral-8x7b", "qwen3-30b-a3b"])
def test_presets(name):
    from llmd_amd.engine.config import get_model_config

    mc = get_model_config(name)
    assert mc.is_moe and mc.model_type in ("mixtral", "qwen3_moe")
