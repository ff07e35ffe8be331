"""OPT family (models/opt.py), the reference's CPU optimized-baseline model
(facebook/opt-125m on docker/Dockerfile.cpu): a randomly initialised HF
``transformers`` OPTForCausalLM is saved as safetensors in the HF layout and
served by our engine; greedy tokens must match HF's own greedy generation and
the first-step logits must agree (no checkpoint download: the HF module is
the reference). GPU: the same with the HIP LayerNorm / attention kernels,
plus LayerNorm kernel numerics against the fp32 reference."""
import numpy as np
import pytest
import torch

from llmd_amd.engine.config import EngineConfig, get_model_config
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams

transformers = pytest.importorskip("transformers")


def _hf_opt(tmp_path, pre_ln=True, proj=0):
    cfg = transformers.OPTConfig(vocab_size=512, hidden_size=256, num_hidden_layers=2, ffn_dim=512,
                                 num_attention_heads=4, max_position_embeddings=512, do_layer_norm_before=pre_ln,
                                 word_embed_proj_dim=proj or 256, dropout=0.0, attention_dropout=0.0,
                                 pad_token_id=1, bos_token_id=2, eos_token_id=2)
    torch.manual_seed(0)
    m = transformers.OPTForCausalLM(cfg).eval()
    with torch.no_grad():  # non-trivial norms and biases so every tensor must be loaded right
        for n, p in m.named_parameters():
            if "layer_norm" in n:
                p.add_(torch.randn_like(p) * 0.2)
            elif n.endswith("bias"):
                p.normal_(0.0, 0.05)
        m = m.to(torch.bfloat16)
    d = tmp_path / "opt"
    m.save_pretrained(d, safe_serialization=True)
    return m, str(d)


def _engine(path, device):
    return LLMEngine(EngineConfig.create(path, device=device, block_size=16 if device == "cpu" else 64,
                                         num_gpu_blocks=64, max_num_batched_tokens=256, max_num_seqs=4,
                                         max_model_len=512, enforce_eager=device == "cpu",
                                         load_format="safetensors", weights_path=path))


def _check(tmp_path, device, pre_ln=True, proj=0):
    hf, path = _hf_opt(tmp_path, pre_ln, proj)
    mc = get_model_config(path)
    assert mc.model_type == "opt" and mc.intermediate_size == 512 and mc.num_key_value_heads == 4
    prompts = [np.random.default_rng(s).integers(3, 500, size=n).tolist() for s, n in ((1, 37), (2, 90))]
    eng = _engine(path, device)
    outs = eng.generate(prompts, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True, logprobs=1))
    hf = hf.to(device)
    for p, o in zip(prompts, outs):
        ids = torch.tensor([p], device=device)
        with torch.no_grad():
            ref = hf.generate(ids, max_new_tokens=6, do_sample=False, min_new_tokens=6)[0, len(p):].tolist()
            lg = hf(ids).logits[0, -1].float().log_softmax(-1)
        # bf16 end to end on both sides: the first token must agree, later ones may
        # flip only at a near-tie of HF's own logits
        assert o.output_token_ids[0] == ref[0]
        assert abs(o.output_logprobs[0] - lg[ref[0]].item()) < 0.15
        agree = sum(a == b for a, b in zip(o.output_token_ids, ref))
        assert agree >= 4, (o.output_token_ids, ref)


def test_opt_matches_hf_cpu(tmp_path):
    _check(tmp_path, "cpu")


def test_opt_post_ln_and_projection_cpu(tmp_path):
    _check(tmp_path, "cpu", pre_ln=False, proj=128)  # opt-350m layout


def test_opt_preset_resolves():
    c = get_model_config("facebook/opt-125m")
    assert (c.model_type, c.hidden_size, c.num_hidden_layers, c.vocab_size) == ("opt", 768, 12, 50272)


@pytest.mark.gpu
def test_opt_matches_hf_gpu(tmp_path):
    _check(tmp_path, "cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("d", [256, 768, 4096])
def test_layer_norm_kernel(d):
    from llmd_amd import ops
    from llmd_amd.ops import reference as ref

    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(37, d, device="cuda", generator=g).bfloat16() * 3 + 1
    r = torch.randn(37, d, device="cuda", generator=g).bfloat16()
    w = torch.randn(d, device="cuda", generator=g).bfloat16()
    b = torch.randn(d, device="cuda", generator=g).bfloat16()
    torch.testing.assert_close(ops.layer_norm(x, w, b, 1e-5).float(), ref.layer_norm(x, w, b, 1e-5).float(),
                               atol=3e-2, rtol=2e-2)
    x1, r1 = x.clone(), r.clone()
    x2, r2 = x.clone(), r.clone()
    ops.fused_add_layer_norm(x1, r1, w, b, 1e-5)
    ref.fused_add_layer_norm(x2, r2, w, b, 1e-5)
    assert torch.equal(r1, r2)
    torch.testing.assert_close(x1.float(), x2.float(), atol=3e-2, rtol=2e-2)
