"""Numerics of every HIP kernel vs the plain PyTorch fp32 reference (GPU only)."""
import math

import pytest
import torch

from llmd_amd import ops
from llmd_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol=2e-2, rtol=2e-2):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=rtol)


def test_native_library_loaded():
    C = ops.native()
    assert C.__file__.endswith(".so")


@pytest.mark.parametrize("T,d", [(1, 4096), (7, 4096), (33, 8192), (5, 2880), (3, 7168), (2, 16384)])
def test_rms_norm(T, d):
    torch.manual_seed(0)
    x = torch.randn(T, d, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(d, device=DEV, dtype=torch.bfloat16)
    _close(ops.rms_norm(x, w, 1e-5), ref.rms_norm(x, w, 1e-5))
    r = torch.randn(T, d, device=DEV, dtype=torch.bfloat16)
    x1, r1 = x.clone(), r.clone()
    ops.fused_add_rms_norm(x1, r1, w, 1e-5)
    x2, r2 = x.clone(), r.clone()
    ref.fused_add_rms_norm(x2, r2, w, 1e-5)
    _close(r1, r2, atol=0, rtol=0)
    _close(x1, x2)


def _cache(nblk, Hkv, bs, D, L=1):
    kv = torch.zeros(nblk, L, 2, Hkv, bs, D, device=DEV, dtype=torch.bfloat16)
    return kv[:, 0, 0], kv[:, 0, 1]


@pytest.mark.parametrize("neox", [True, False])
@pytest.mark.parametrize("Hq,Hkv,D,rot,bs", [(32, 8, 128, 128, 16), (64, 8, 64, 64, 64), (8, 2, 128, 64, 32)])
def test_rope_cache(neox, Hq, Hkv, D, rot, bs):
    torch.manual_seed(1)
    T = 37
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    cs = ref.rope_cos_sin(rot, 4096, 500000.0, device=DEV)
    nblk = 16
    slots = torch.randperm(nblk * bs, device=DEV)[:T]
    slots[3] = -1
    k1, v1 = _cache(nblk, Hkv, bs, D, L=3)
    k2, v2 = _cache(nblk, Hkv, bs, D, L=3)
    a, b = qkv.clone(), qkv.clone()
    ops.rope_cache(a, pos, cs, Hq, Hkv, D, slots, k1, v1, neox)
    ref.rope_cache(b, pos, cs, Hq, Hkv, D, slots, k2, v2, neox)
    _close(a[:, : Hq * D], b[:, : Hq * D])
    _close(k1, k2)
    _close(v1, v2, atol=0, rtol=0)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gated_act(mode):
    torch.manual_seed(2)
    x = torch.randn(19, 2 * 1024, device=DEV, dtype=torch.bfloat16) * 3
    _close(ops.gated_act(x, mode), ref.gated_act(x, mode))


def _paged_setup(lens, Hkv, D, bs, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    nb_per = [(L + bs - 1) // bs for L in lens]
    total = sum(nb_per) + 3
    kc, vc = _cache(total, Hkv, bs, D, L=2)
    kc.copy_(torch.randn(kc.shape, generator=g).to(DEV, torch.bfloat16))
    vc.copy_(torch.randn(vc.shape, generator=g).to(DEV, torch.bfloat16))
    perm = torch.randperm(total, generator=g)
    width = max(nb_per) + 2
    bt = torch.zeros(len(lens), width, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nb_per):
        bt[i, :n] = perm[o : o + n].int()
        o += n
    return kc, vc, bt.to(DEV)


@pytest.mark.parametrize("Hq,Hkv,D", [(64, 8, 128), (32, 8, 128), (8, 8, 128), (64, 8, 64), (16, 1, 128), (40, 2, 128)])
@pytest.mark.parametrize("bs", [16, 64])
def test_paged_decode(Hq, Hkv, D, bs):
    lens = [1, 63, 64, 65, 300, 1029, 4999]
    kc, vc, bt = _paged_setup(lens, Hkv, D, bs)
    B = len(lens)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    r = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale)
    for split in [None, (64, 79), (4096, 2), (5056, 1)]:
        o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, split=split, max_ctx=max(lens))
        _close(o, r)


def test_paged_decode_window_sinks():
    Hq, Hkv, D, bs = 64, 8, 64, 16
    lens = [5, 128, 129, 700]
    kc, vc, bt = _paged_setup(lens, Hkv, D, bs, seed=3)
    q = torch.randn(len(lens), Hq * D, device=DEV, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    sinks = torch.randn(Hq, device=DEV)
    for window in [0, 128]:
        r = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, 0.125, window, sinks)
        for split in [None, (64, 11)]:
            o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, 0.125, window, sinks, split=split, max_ctx=700)
            _close(o, r)


@pytest.mark.parametrize("Hq,Hkv,D", [(64, 8, 128), (32, 8, 128), (8, 8, 128), (64, 8, 64), (16, 8, 128)])
@pytest.mark.parametrize("bs", [16, 64])
def test_paged_prefill(Hq, Hkv, D, bs):
    # (q_len, ctx_len): fresh prompts, chunked prefill over cached prefix, tiny
    shapes = [(1, 1), (37, 37), (200, 200), (130, 1000), (64, 64), (513, 700)]
    ctx = [c for _, c in shapes]
    kc, vc, bt = _paged_setup(ctx, Hkv, D, bs, seed=5)
    ql = [a for a, _ in shapes]
    qs = [0]
    for a in ql[:-1]:
        qs.append(qs[-1] + a)
    T = sum(ql)
    q = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    args = [torch.tensor(x, dtype=torch.int32, device=DEV) for x in (qs, ql, ctx)]
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, 1 / math.sqrt(D))
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, 1 / math.sqrt(D))
    _close(o, r)


def test_paged_prefill_window_sinks():
    Hq, Hkv, D, bs = 64, 8, 64, 16
    shapes = [(300, 300), (77, 500)]
    ctx = [c for _, c in shapes]
    kc, vc, bt = _paged_setup(ctx, Hkv, D, bs, seed=6)
    ql = [a for a, _ in shapes]
    qs = [0, ql[0]]
    q = torch.randn(sum(ql), Hq * D, device=DEV, dtype=torch.bfloat16)
    sinks = torch.randn(Hq, device=DEV)
    args = [torch.tensor(x, dtype=torch.int32, device=DEV) for x in (qs, ql, ctx)]
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, 0.125, 128, sinks)
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, 0.125, 128, sinks)
    _close(o, r)


def test_sample_greedy_and_logprob():
    torch.manual_seed(7)
    logits = torch.randn(9, 128256, device=DEV).to(torch.bfloat16)
    ids, lp = ops.sample(logits, want_logprob=True)
    assert torch.equal(ids, logits.float().argmax(-1))
    ref_lp = torch.log_softmax(logits.float(), -1).gather(-1, ids[:, None]).squeeze(-1)
    _close(lp, ref_lp, atol=1e-3, rtol=1e-3)


def test_sample_temperature_distribution():
    V = 8
    logits = torch.tensor([[0.0, 1.0, 2.0, 0.5, -1.0, 0.0, 3.0, 1.5]], device=DEV).repeat(20000, 1)
    temps = torch.full((20000,), 0.7, device=DEV)
    seeds = torch.arange(20000, device=DEV, dtype=torch.int64) * 7919 + 3
    ids, _ = ops.sample(logits, temps, seeds)
    freq = torch.bincount(ids, minlength=V).float() / ids.numel()
    p = torch.softmax(logits[0] / 0.7, -1)
    assert (freq - p).abs().max() < 0.015


def test_topk_topp_mask():
    torch.manual_seed(8)
    B, V = 6, 5000
    x = torch.randn(B, V, device=DEV)
    topk = torch.tensor([0, 1, 5, 50, 4999, 17], dtype=torch.int32, device=DEV)
    topp = torch.tensor([0.9, 1.0, 0.5, 0.95, 0.1, 1.0], device=DEV)
    temps = torch.tensor([1.0, 0.5, 1.0, 2.0, 1.0, 1.0], device=DEV)
    a = ops.topk_topp_mask(x.clone(), topk, None, temps)
    b = ref.topk_topp_mask(x.clone(), topk, None, temps)
    assert torch.equal(torch.isinf(a), torch.isinf(b))
    a = ops.topk_topp_mask(x.clone(), None, topp, temps)
    b = ref.topk_topp_mask(x.clone(), None, topp, temps)
    assert torch.equal(torch.isinf(a), torch.isinf(b))
