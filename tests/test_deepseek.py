"""DeepSeek (MLA + shared-expert MoE): the engine's absorbed-MLA path over the
paged latent cache must reproduce a plain non-absorbed MLA forward (per-head
K/V expanded from the latent), on CPU; GPU: the HIP latent-attention and
rope/cache kernels against their fp32 references, and the engine on MI355X."""
import math

import numpy as np
import pytest
import torch

from llmd_amd import ops
from llmd_amd.ops import reference as ref
from llmd_amd.engine.request import SamplingParams
from tests.test_engine import _prompts, make_engine


def _rot_gptj(x, cos, sin):
    x0, x1 = x[..., 0::2], x[..., 1::2]
    return torch.stack([x0 * cos - x1 * sin, x0 * sin + x1 * cos], -1).flatten(-2)


def plain_forward_ds(model, ids):
    cfg = model.cfg
    dev = model.embed.weight.device
    x = torch.nn.functional.embedding(torch.tensor(ids, device=dev), model.embed.weight)
    T = len(ids)
    pos = torch.arange(T, device=dev)
    cs = model.cos_sin[pos].float()
    cos, sin = cs[:, :32], cs[:, 32:]
    residual = None
    mask = torch.ones(T, T, dtype=torch.bool, device=dev).tril()
    for layer in model.layers:
        if residual is None:
            residual = x.clone()
            x = ref.rms_norm(x, layer.input_layernorm.weight, cfg.rms_norm_eps)
        else:
            ref.fused_add_rms_norm(x, residual, layer.input_layernorm.weight, cfg.rms_norm_eps)
        a = layer.attn
        H = a.H
        lin = torch.nn.functional.linear
        if a.q_lora:
            q = lin(ref.rms_norm(lin(x, a.q_a.weight), a.q_a_norm.weight, cfg.rms_norm_eps), a.q_b.weight)
        else:
            q = lin(x, a.q_proj.weight)
        q = q.float().view(T, H, 192)
        kv = lin(x, a.kv_a.weight)
        c = ref.rms_norm(kv[:, :512].contiguous(), a.kv_a_norm.weight, cfg.rms_norm_eps).float()
        k_pe = _rot_gptj(kv[:, 512:].float(), cos, sin)                      # [T, 64]
        q_pe = _rot_gptj(q[:, :, 128:], cos[:, None], sin[:, None])         # [T, H, 64]
        w = a.kv_b.float().view(H, 256, 512)
        k_nope = torch.einsum("tc,hdc->thd", c, w[:, :128])                  # [T, H, 128]
        v = torch.einsum("tc,hdc->thd", c, w[:, 128:])
        s = (torch.einsum("thd,shd->hts", q[:, :, :128], k_nope) +
             torch.einsum("thd,sd->hts", q_pe, k_pe)) * a.scale
        p = torch.softmax(s.masked_fill(~mask, float("-inf")), -1)
        o = torch.einsum("hts,shd->thd", p, v).reshape(T, H * 128).to(x.dtype)
        x = lin(o, a.o_proj.weight)
        ref.fused_add_rms_norm(x, residual, layer.post_attention_layernorm.weight, cfg.rms_norm_eps)
        x = layer.mlp(x)
    ref.fused_add_rms_norm(x, residual, model.norm.weight, cfg.rms_norm_eps)
    return torch.nn.functional.linear(x[-1:], model.lm_head.weight)[0, : cfg.vocab_size].float()


def _greedy(model, prompt, n):
    ids, out = list(prompt), []
    for _ in range(n):
        t = int(plain_forward_ds(model, ids).argmax())
        out.append(t)
        ids.append(t)
    return out


def test_deepseek_engine_matches_plain_mla():
    eng = make_engine(model="tiny-deepseek")
    prompts = _prompts(9, [7, 70, 33])
    reqs = eng.generate(prompts, SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True))
    agree = total = 0
    for p, r in zip(prompts, reqs):
        g = _greedy(eng.runner.model, p, 5)
        assert r.output_token_ids[0] == g[0]
        agree += sum(int(a == b) for a, b in zip(r.output_token_ids, g))
        total += len(g)
    assert agree / total >= 0.8


def test_mla_reference_matches_expanded_attention():
    torch.manual_seed(0)
    H, bs, L = 4, 16, 40
    cache = torch.randn(4, bs, 576, dtype=torch.bfloat16)
    bt = torch.tensor([[2, 0, 3]], dtype=torch.int32)
    q = torch.randn(3, H * 576, dtype=torch.bfloat16)
    rows = torch.zeros(3, dtype=torch.int32)
    lens = torch.tensor([L, 17, 1], dtype=torch.int32)
    out = ref.mla_attention(q, cache, bt, rows, lens, H, 0.1)
    flat = torch.cat([cache[2], cache[0], cache[3]]).float()
    for r in range(3):
        kv = flat[: int(lens[r])]
        p = torch.softmax(q[r].float().view(H, 576) @ kv.T * 0.1, -1)
        assert torch.allclose(out[r].float().view(H, 512), (p @ kv[:, :512]), atol=2e-2)


def test_deepseek_hf_roundtrip_and_tp_ep_specs(tmp_path):
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, load_weights, save_safetensors
    from llmd_amd.engine.config import get_model_config

    cfg = get_model_config("tiny-deepseek")
    m = build_model(cfg, device="cpu", max_pos=600)
    sd = export_hf(m)
    assert "model.layers.1.mlp.experts.3.up_proj.weight" in sd and "model.layers.0.mlp.gate_proj.weight" in sd
    path = str(tmp_path / "ds.safetensors")
    save_safetensors(sd, path)
    torch.manual_seed(1)
    m2 = build_model(cfg, device="cpu", max_pos=600)
    load_weights(m2, path)
    for (n1, a), (n2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), n1


@pytest.mark.gpu
def test_mla_kernel_matches_reference():
    torch.manual_seed(0)
    dev = "cuda"
    for H, lens, bs in ((20, [1, 63, 64, 65, 300], 16), (128, [1000, 4096, 7], 64), (16, [2500], 64),
                      (128, [1, 65, 300], 16), (64, [777, 64, 129], 64)):
        nb_per = max(math.ceil(L / bs) for L in lens)
        nseq = len(lens)
        nb = nseq * nb_per + 3
        pool = torch.randn(nb, 2, bs, 576, dtype=torch.bfloat16, device=dev)  # non-contiguous layer view
        cache = pool[:, 1]
        bt = torch.stack([torch.randperm(nb, device=dev)[:nb_per] for _ in range(nseq)]).int()
        R = nseq
        q = torch.randn(R, H * 576, dtype=torch.bfloat16, device=dev)
        rows = torch.arange(R, dtype=torch.int32, device=dev)
        ln = torch.tensor(lens, dtype=torch.int32, device=dev)
        scale = 576 ** -0.5
        want = ref.mla_attention(q, cache, bt, rows, ln, H, scale)
        for split in (None, (64, math.ceil(max(lens) / 64)), (max(64, math.ceil(max(lens) / 64) * 64), 1)):
            got = ops.mla_attention(q, cache, bt, rows, ln, H, scale, split=split)
            err = (got.float() - want.float()).abs().max().item()
            assert err < 2e-2, (H, lens, split, err)
        # device-side split size (hipGraph replay): a 16k-key plan's 8 splits re-sized to the rows
        dyn = torch.tensor([max(256, math.ceil(max(lens) / (64 * 8)) * 64)], dtype=torch.int32, device=dev)
        got = ops.mla_attention(q, cache, bt, rows, ln, H, scale, split=(16384, 8), split_dev=dyn)
        err = (got.float() - want.float()).abs().max().item()
        assert err < 2e-2, (H, lens, "split_dev", err)


@pytest.mark.gpu
def test_mla_prefill_rows_and_rope_cache_kernel():
    torch.manual_seed(1)
    dev = "cuda"
    T, H, bs = 37, 20, 16
    cos_sin = ops.rope_cos_sin(64, 512, 10000.0, None, device=dev)
    q = torch.randn(T, H * 192, dtype=torch.bfloat16, device=dev)
    kv = torch.randn(T, 576, dtype=torch.bfloat16, device=dev)
    pos = torch.arange(100, 100 + T, device=dev)
    slots = torch.arange(T, device=dev) + 5
    slots[3] = -1
    cache_a = torch.zeros(8, bs, 576, dtype=torch.bfloat16, device=dev)
    cache_b = torch.zeros_like(cache_a)
    ql_a = torch.zeros(T, H * 576, dtype=torch.bfloat16, device=dev)
    ql_b = torch.zeros_like(ql_a)
    ops.mla_rope_cache(q, ql_a, kv[:, :512], kv[:, 512:], pos, cos_sin, H, slots, cache_a)
    ref.mla_rope_cache(q, ql_b, kv[:, :512], kv[:, 512:], pos, cos_sin, H, slots, cache_b)
    assert (ql_a.float() - ql_b.float()).abs().max().item() < 2e-2
    assert (cache_a.float() - cache_b.float()).abs().max().item() < 2e-2
    # causal prefill rows: token i of a 37-token chunk at context offset 0 sees i+1 keys
    bt = torch.arange(8, dtype=torch.int32, device=dev)[None]
    rows = torch.zeros(T, dtype=torch.int32, device=dev)
    ln = torch.arange(1, T + 1, dtype=torch.int32, device=dev)
    qq = torch.randn(T, H * 576, dtype=torch.bfloat16, device=dev)
    got = ops.mla_attention(qq, cache_a, bt, rows, ln, H, 0.05)
    want = ref.mla_attention(qq, cache_a, bt, rows, ln, H, 0.05)
    assert (got.float() - want.float()).abs().max().item() < 2e-2


@pytest.mark.gpu
def test_deepseek_engine_gpu():
    eng = make_engine(device="cuda", num_gpu_blocks=128, max_num_batched_tokens=256, model="tiny-deepseek",
                      max_num_seqs=8)
    prompts = _prompts(3, [5, 120, 40])
    reqs = eng.generate(prompts, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))
    model = eng.runner.model
    for p, r in zip(prompts, reqs):
        assert r.output_token_ids[0] == _greedy(model, p, 1)[0]
    assert np.isfinite(eng.metrics.n_gen)
