"""FP8 (OCP e4m3fn) KV cache: HIP rope+cache write, decode and prefill attention
vs the fp32 reference over the same dequantised cache (GPU), and the engine
running end to end with --kv-cache-dtype fp8 (CPU reference ops)."""
import math

import pytest
import torch

from llmd_amd import ops
from llmd_amd.ops import reference as ref

F8 = torch.float8_e4m3fn


def _close(a, b, atol=3e-2, rtol=3e-2):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=rtol)


def _cache(nblk, Hkv, bs, D, dev, L=2, dtype=F8):
    kv = torch.zeros(nblk, L, 2, Hkv, bs, D, device=dev, dtype=dtype)
    return kv[:, 0, 0], kv[:, 0, 1]


def _paged(lens, Hkv, D, bs, dev, seed=0, ks=1.0, vs=1.0):
    g = torch.Generator().manual_seed(seed)
    nb_per = [(L + bs - 1) // bs for L in lens]
    total = sum(nb_per) + 3
    kc, vc = _cache(total, Hkv, bs, D, dev)
    kc.copy_(ref.to_cache(torch.randn(kc.shape, generator=g) * 2, F8, ks).to(dev))
    vc.copy_(ref.to_cache(torch.randn(vc.shape, generator=g) * 2, F8, vs).to(dev))
    perm = torch.randperm(total, generator=g)
    bt = torch.zeros(len(lens), max(nb_per) + 2, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nb_per):
        bt[i, :n] = perm[o:o + n].int()
        o += n
    return kc, vc, bt.to(dev)


def test_reference_fp8_cache_roundtrip():
    x = torch.tensor([0.0, 1.0, -3.5, 2000.0, -1000.0, 0.0117])
    c = ref.to_cache(x, F8, 2.0)
    back = c.float() * 2.0
    assert back[3].item() == 448.0 * 2 and back[4].item() == -448.0 * 2  # saturated, not NaN
    assert abs(back[2].item() + 3.5) < 1e-6


def test_engine_fp8_kv_cpu():
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    outs = {}
    for kvd in ("auto", "fp8"):
        cfg = EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                                  max_num_batched_tokens=256, max_num_seqs=4, max_model_len=512,
                                  kv_cache_dtype=kvd)
        eng = LLMEngine(cfg, capture_graphs=False)
        assert eng.runner.kv.dtype == (F8 if kvd == "fp8" else torch.bfloat16)
        reqs = eng.generate([list(range(3, 40)), [7] * 20], SamplingParams(max_tokens=6, temperature=0.0,
                                                                           ignore_eos=True))
        outs[kvd] = [r.output_token_ids for r in reqs]
    assert all(len(o) == 6 for o in outs["fp8"])
    # fp8 KV perturbs logits slightly; the first greedy token matches on a random-init model
    assert [o[0] for o in outs["fp8"]] == [o[0] for o in outs["auto"]]


@pytest.mark.gpu
@pytest.mark.parametrize("neox", [True, False])
def test_rope_cache_fp8(neox):
    dev = "cuda"
    torch.manual_seed(1)
    Hq, Hkv, D, rot, bs, T = 32, 8, 128, 128, 16, 37
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16) * 3
    pos = torch.randint(0, 4000, (T,), device=dev)
    cs = ref.rope_cos_sin(rot, 4096, 500000.0, device=dev)
    slots = torch.randperm(16 * bs, device=dev)[:T]
    slots[3] = -1
    k1, v1 = _cache(16, Hkv, bs, D, dev)
    k2, v2 = _cache(16, Hkv, bs, D, dev)
    a, b = qkv.clone(), qkv.clone()
    ops.rope_cache(a, pos, cs, Hq, Hkv, D, slots, k1, v1, neox, 0.5, 2.0)
    ref.rope_cache(b, pos, cs, Hq, Hkv, D, slots, k2, v2, neox, 0.5, 2.0)
    _close(a[:, :Hq * D], b[:, :Hq * D], atol=2e-2, rtol=2e-2)
    # one fp8 ulp of slack (bf16 rounding of the rotated value can flip the fp8 rounding)
    _close(k1.float(), k2.float(), atol=0.25, rtol=0.07)
    _close(v1.float(), v2.float(), atol=0, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("Hq,Hkv,D", [(64, 8, 128), (32, 8, 64), (8, 8, 128)])
def test_paged_decode_fp8(Hq, Hkv, D):
    dev = "cuda"
    lens = [1, 65, 300, 1029, 4999]
    ks, vs = 0.75, 1.5
    kc, vc, bt = _paged(lens, Hkv, D, 64, dev, ks=ks, vs=vs)
    q = torch.randn(len(lens), (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=dev)
    scale = 1 / math.sqrt(D)
    r = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, k_scale=ks, v_scale=vs)
    for split in [None, (64, 79), (5056, 1)]:
        o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, split=split, max_ctx=max(lens),
                             k_scale=ks, v_scale=vs)
        _close(o, r)


@pytest.mark.gpu
def test_paged_decode_fp8_window_sinks():
    dev = "cuda"
    Hq, Hkv, D = 64, 8, 64
    lens = [5, 129, 700]
    kc, vc, bt = _paged(lens, Hkv, D, 16, dev, seed=3)
    q = torch.randn(len(lens), Hq * D, device=dev, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=dev)
    sinks = torch.randn(Hq, device=dev)
    r = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, 0.125, 128, sinks)
    o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, 0.125, 128, sinks, split=(64, 11), max_ctx=700)
    _close(o, r)


@pytest.mark.gpu
@pytest.mark.parametrize("via_bf16", [True, False])
@pytest.mark.parametrize("Hq,Hkv,D", [(64, 8, 128), (32, 8, 64), (16, 8, 128)])
def test_paged_prefill_fp8(Hq, Hkv, D, via_bf16, monkeypatch):
    """fp8 KV prefill: through a bf16 copy of the step's blocks + the bf16 v2 kernel (default) and
    the fp8 v1 kernel, both against the fp32 reference on the same scaled caches."""
    monkeypatch.setattr(ops, "PREFILL_FP8_VIA_BF16", via_bf16)
    dev = "cuda"
    shapes = [(1, 1), (37, 37), (200, 200), (130, 1000), (513, 700)]
    ctx = [c for _, c in shapes]
    ks, vs = 1.25, 0.5
    kc, vc, bt = _paged(ctx, Hkv, D, 64, dev, seed=5, ks=ks, vs=vs)
    ql = [a for a, _ in shapes]
    qs = [0]
    for a in ql[:-1]:
        qs.append(qs[-1] + a)
    q = torch.randn(sum(ql), (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    args = [torch.tensor(x, dtype=torch.int32, device=dev) for x in (qs, ql, ctx)]
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, 1 / math.sqrt(D), k_scale=ks, v_scale=vs)
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, 1 / math.sqrt(D), k_scale=ks, v_scale=vs)
    _close(o, r)


def test_kv_dequant_gather_cpu_widens_exactly():
    """The CPU form of the gather (the GPU kernel's contract): entry e of the table -> row e, e4m3
    widened exactly, padding entries (-1) -> block 0, identity table over the copy."""
    torch.manual_seed(0)
    kc = (torch.randn(6, 2, 16, 64) * 3).to(ops.FP8)
    vc = (torch.randn(6, 2, 16, 64) * 3).to(ops.FP8)
    bt = torch.tensor([[4, 1, -1], [2, 5, 0]], dtype=torch.int32)
    kd, vd, t2 = ops.kv_dequant_gather(kc, vc, bt)
    assert kd.dtype == torch.bfloat16 and kd.shape == (6, 2, 16, 64)
    assert torch.equal(kd[0].float(), kc[4].float()) and torch.equal(vd[4].float(), vc[5].float())
    assert torch.equal(kd[2].float(), kc[0].float())
    assert torch.equal(t2, torch.arange(6, dtype=torch.int32).view(2, 3))


def test_fp8_linear_cpu_matches_fp32():
    torch.manual_seed(0)
    x = torch.randn(5, 64, dtype=torch.bfloat16)
    w = torch.randn(48, 64, dtype=torch.bfloat16) * 0.05
    wq, ws = ops.quant_fp8_weight(w)
    y = ops.fp8_linear(x, wq, ws)
    r = x.float() @ w.float().t()
    assert y.shape == (5, 48)
    # W8A8 e4m3: ~2 x 2^-4 relative error per product, averaged over K
    assert (y.float() - r).abs().max() < 0.08 * r.abs().max()


def test_engine_fp8_w8a8_cpu():
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    cfg = EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                              max_num_batched_tokens=256, max_num_seqs=4, max_model_len=512,
                              quantization="fp8", kv_cache_dtype="fp8")
    eng = LLMEngine(cfg, capture_graphs=False)
    qkv = eng.runner.model.layers[0].qkv
    if qkv is not None:
        assert qkv.weight.dtype == F8 and qkv.weight_scale.shape == (1, qkv.weight.shape[0])
    reqs = eng.generate([list(range(3, 30))], SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    assert len(reqs[0].output_token_ids) == 4


@pytest.mark.gpu
@pytest.mark.parametrize("T,K,N", [(1, 8192, 10240), (64, 8192, 8192), (300, 4096, 28672), (2048, 7168, 4096)])
def test_fp8_linear_gpu(T, K, N):
    torch.manual_seed(0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    wq, ws = ops.quant_fp8_weight(w)
    xq, xs = ops.quant_fp8_rows(x)
    rq, rs = ops.quant_fp8_rows(x.cpu())
    torch.testing.assert_close(xs.cpu(), rs, rtol=1e-6, atol=0)
    assert (xq.cpu().float() - rq.float()).abs().max() <= 32  # at most 1 ulp at the top of the range
    y = ops.fp8_linear(x, wq, ws)
    r = (xq.float() * xs) @ (wq.float() * ws.view(-1, 1)).t()
    torch.testing.assert_close(y.float(), r, atol=2e-2 * r.abs().max().item(), rtol=2e-2)


def test_moe_fp8_block_quant_cpu():
    torch.manual_seed(0)
    E, N, K = 3, 200, 272
    w = torch.randn(E, N, K) * 0.05
    q, s = ops.quant_fp8_block_weight(w)
    assert q.shape == (E, N, K) and s.shape == (E, 2, 3)
    back = ops.dequant_fp8_block_weight(q, s)
    assert (back - w).abs().max() < 0.07 * w.abs().max()
    x = torch.randn(5, 300).to(torch.bfloat16)
    xq, xs = ops.quant_fp8_groups(x)
    assert xs.shape == (5, 3)
    xd = xq.float() * xs.repeat_interleave(128, 1)[:, :300]
    assert (xd - x.float()).abs().max() < 0.07 * x.float().abs().max()


def test_engine_fp8_moe_cpu():
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    cfg = EngineConfig.create("tiny-gpt-oss", device="cpu", block_size=16, num_gpu_blocks=64,
                              max_num_batched_tokens=256, max_num_seqs=4, max_model_len=512, quantization="fp8")
    eng = LLMEngine(cfg, capture_graphs=False)
    mlp = eng.runner.model.layers[0].mlp
    assert mlp.w1.dtype == F8 and mlp.w1_scale.dim() == 3
    reqs = eng.generate([list(range(3, 30))], SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
    assert len(reqs[0].output_token_ids) == 3


@pytest.mark.gpu
@pytest.mark.parametrize("T,E,k,d,F,act", [(1, 8, 2, 256, 128, 0), (37, 32, 4, 2880, 2880, 2),
                                           (100, 16, 8, 7168, 2048, 0), (64, 128, 4, 2880, 2880, 2)])
def test_moe_experts_fp8_gpu(T, E, k, d, F, act):
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.03
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.03
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    w2q, w2s = ops.quant_fp8_block_weight(w2)
    logits = torch.randn(T, E, device=dev)
    ids, wts = ops.moe_topk(logits, k, scoring=0)
    # group quant matches the CPU reference
    xq, xs = ops.quant_fp8_groups(x)
    rq, rs = ops.quant_fp8_groups(x.cpu())
    torch.testing.assert_close(xs.cpu(), rs, rtol=1e-6, atol=0)
    y = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act)
    r = ops.moe_experts_fp8(x.cpu(), ids.cpu(), wts.cpu(), w1q.cpu(), w1s.cpu(), w2q.cpu(), w2s.cpu(), act)
    err = (y.float().cpu() - r.float()).abs().max().item()
    assert err < 0.06 * r.float().abs().max().item() + 1e-3, err
    if d % 128 or F % 128:  # K padded to whole 128-wide steps (quantize_fp8 on GPU): the v2 kernel path
        c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
        yp = ops.moe_experts_fp8(x, ids, wts, ops.pad_fp8_k(w1q, c128(d)), w1s, ops.pad_fp8_k(w2q, c128(F)), w2s,
                                 act)
        errp = (yp.float().cpu() - r.float()).abs().max().item()
        assert errp < 0.06 * r.float().abs().max().item() + 1e-3, errp


@pytest.mark.gpu
@pytest.mark.parametrize("T,E,k,d,F,act,skew", [(512, 4, 4, 1024, 1024, 2, False), (600, 16, 8, 1024, 256, 0, True),
                                                (700, 64, 4, 384, 256, 2, True), (5, 8, 2, 256, 128, 0, False)])
def test_moe_fp8_prefill_tiles_gpu(T, E, k, d, F, act, skew, monkeypatch):
    """256-row expert tiles (moe_gemm3_fp8_kernel, E8M0 hardware scales) vs the
    64-row kernel and the CPU reference, incl. experts with no rows, partial
    tiles (valid-row prefix) and multi-tile experts."""
    torch.manual_seed(1)
    dev = "cuda"
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.03
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.03
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    w1q, w1s = ops.quant_fp8_block_weight(w1)
    w2q, w2s = ops.quant_fp8_block_weight(w2)
    assert torch.equal(ops.pow2_ceil(w1s), w1s)  # E8M0-exact block scales
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    logits = torch.randn(T, E, device=dev)
    if skew:  # a quarter of the experts take most tokens, the last ones (almost) none
        logits[:, : E // 4] += 2.0
        logits[:, -2:] -= 8.0
    ids, wts = ops.moe_topk(logits, k, scoring=0)
    monkeypatch.setattr(ops, "MOE_V3", True)
    monkeypatch.setattr(ops, "MOE_V3_MIN_ROWS", 0)
    y3 = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1)
    monkeypatch.setattr(ops, "MOE_V3", False)
    y2 = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1)
    r = ops.moe_experts_fp8(x.cpu(), ids.cpu(), wts.cpu(), w1q.cpu()[..., :d], w1s.cpu(), w2q.cpu()[..., :F],
                            w2s.cpu(), act, b1=b1.cpu())
    m = r.float().abs().max().item()
    assert torch.isfinite(y3).all()
    assert (y3.float().cpu() - r.float()).abs().max().item() < 0.06 * m + 1e-3
    assert (y3.float() - y2.float()).abs().max().item() < 0.02 * m + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("T,E,k,d,F,act,skew", [(512, 4, 4, 1024, 1024, 2, False), (600, 16, 8, 1024, 256, 0, True),
                                                (800, 16, 4, 2880, 2880, 2, False), (300, 8, 8, 7168, 2048, 0, True),
                                                (5, 8, 2, 256, 128, 0, False)])
@pytest.mark.parametrize("tile", ["256", "192"])
def test_moe_fp8_v4_gpu(T, E, k, d, F, act, skew, tile, monkeypatch):
    """The v4 block-fp8 grouped GEMM (csrc/ops/moe4.hip moe_gemm4_fp8_kernel: 4-wave PGR2 tiles,
    A rows and their act scales gathered by the LDS-DMA, scaled 32x32x64 MFMA) vs the v3 256-row
    kernel and the CPU reference: gpt-oss widths (partial column tiles), K = 7168 (56 k-blocks),
    empty and multi-tile experts, biases."""
    torch.manual_seed(3)
    dev = "cuda"
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1q, w1s = ops.quant_fp8_block_weight(torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.03)
    w2q, w2s = ops.quant_fp8_block_weight(torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.03)
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    b2 = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.1
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    logits = torch.randn(T, E, device=dev)
    if skew:
        logits[:, : E // 4] += 2.0
        logits[:, -2:] -= 8.0
    ids, wts = ops.moe_topk(logits, k, scoring=0)
    monkeypatch.setattr(ops, "MOE_V3", True)
    monkeypatch.setattr(ops, "MOE_V3_MIN_ROWS", 0)
    monkeypatch.setattr(ops, "MOE_FUSED_QUANT", False)
    monkeypatch.setattr(ops, "MOE_FP8_V4", False)
    y3 = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1, b2=b2)
    monkeypatch.setattr(ops, "MOE_FP8_V4", True)
    monkeypatch.setattr(ops, "MOE4_TILE", tile)
    y4 = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1, b2=b2)
    r = ops.moe_experts_fp8(x.cpu(), ids.cpu(), wts.cpu(), w1q.cpu()[..., :d], w1s.cpu(), w2q.cpu()[..., :F],
                            w2s.cpu(), act, b1=b1.cpu(), b2=b2.cpu())
    m = r.float().abs().max().item()
    assert torch.isfinite(y4).all()
    assert (y4.float().cpu() - r.float()).abs().max().item() < 0.06 * m + 1e-3
    assert (y4.float() - y3.float()).abs().max().item() < 0.02 * m + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("T,E,k,d,F,act,skew", [(512, 4, 4, 1024, 1024, 2, False), (600, 16, 8, 1024, 256, 0, True),
                                                (800, 16, 4, 2880, 2880, 2, False), (300, 8, 8, 7168, 2048, 0, True),
                                                (5, 8, 2, 256, 128, 0, False)])
@pytest.mark.parametrize("tile", ["256", "192"])
def test_moe_fp8_v8_gpu(T, E, k, d, F, act, skew, tile, monkeypatch):
    """The v8 block-fp8 grouped GEMM (csrc/ops/moe8.hip: v4's tile loop made persistent - the
    LDS-DMA stream crosses tile edges, the epilogue stores from the accumulators) vs the v4 kernel on
    the same tiles and the CPU reference: gpt-oss widths (partial column tiles, a 2880 = 22.5 x 128 N),
    K = 7168 (56 k-blocks), empty and multi-tile experts, biases, both tile heights."""
    torch.manual_seed(3)
    dev = "cuda"
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1q, w1s = ops.quant_fp8_block_weight(torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.03)
    w2q, w2s = ops.quant_fp8_block_weight(torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.03)
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    b2 = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.1
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    logits = torch.randn(T, E, device=dev)
    if skew:
        logits[:, : E // 4] += 2.0
        logits[:, -2:] -= 8.0
    ids, wts = ops.moe_topk(logits, k, scoring=0)
    monkeypatch.setattr(ops, "MOE_V3", True)
    monkeypatch.setattr(ops, "MOE_V3_MIN_ROWS", 0)
    monkeypatch.setattr(ops, "MOE_FUSED_QUANT", False)
    monkeypatch.setattr(ops, "MOE_FP8_V4", True)
    monkeypatch.setattr(ops, "MOE4_TILE", tile)
    monkeypatch.setattr(ops, "MOE_FP8_V8", False)
    y4 = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1, b2=b2)
    monkeypatch.setattr(ops, "MOE_FP8_V8", True)
    y8 = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1, b2=b2)
    r = ops.moe_experts_fp8(x.cpu(), ids.cpu(), wts.cpu(), w1q.cpu()[..., :d], w1s.cpu(), w2q.cpu()[..., :F],
                            w2s.cpu(), act, b1=b1.cpu(), b2=b2.cpu())
    m = r.float().abs().max().item()
    assert torch.isfinite(y8).all()
    assert (y8.float().cpu() - r.float()).abs().max().item() < 0.06 * m + 1e-3
    assert (y8.float() - y4.float()).abs().max().item() < 0.02 * m + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("T,E,k,d,F,act,skew", [(64, 16, 4, 1024, 512, 0, False), (100, 32, 8, 2880, 2880, 2, False),
                                                (7, 8, 2, 7168, 2048, 0, True), (256, 128, 4, 2880, 2880, 2, True)])
def test_moe_fp8_t64_gpu(T, E, k, d, F, act, skew, monkeypatch):
    """Decode-sized steps on 64-row persistent tiles (moe8.hip with MB = 1, LLMD_MOE_FP8_T64) vs the
    64-row weight-streaming kernel and the CPU reference: partial column tiles, K = 7168, empty experts."""
    torch.manual_seed(4)
    dev = "cuda"
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1q, w1s = ops.quant_fp8_block_weight(torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.03)
    w2q, w2s = ops.quant_fp8_block_weight(torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.03)
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    b2 = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.1
    w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
    logits = torch.randn(T, E, device=dev)
    if skew:
        logits[:, : E // 4] += 2.0
        logits[:, -2:] -= 8.0
    ids, wts = ops.moe_topk(logits, k, scoring=0)
    assert T * k < ops.MOE_V3_MIN_ROWS * E  # a decode-sized step
    monkeypatch.setattr(ops, "MOE_FUSED_QUANT", False)
    monkeypatch.setattr(ops, "MOE_FP8_T64", False)
    ys = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1, b2=b2)
    monkeypatch.setattr(ops, "MOE_FP8_T64", True)
    yt = ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act, b1=b1, b2=b2)
    r = ops.moe_experts_fp8(x.cpu(), ids.cpu(), wts.cpu(), w1q.cpu()[..., :d], w1s.cpu(), w2q.cpu()[..., :F],
                            w2s.cpu(), act, b1=b1.cpu(), b2=b2.cpu())
    m = r.float().abs().max().item()
    assert torch.isfinite(yt).all()
    assert (yt.float().cpu() - r.float()).abs().max().item() < 0.06 * m + 1e-3
    assert (yt.float() - ys.float()).abs().max().item() < 0.02 * m + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("tile", [256, 192, 64])
def test_moe_gemm8_fp8_kernel_matches_fp32(mode, tile):
    """One v8 grouped GEMM on its own against the fp32 PyTorch oracle of the same op (dequantised
    operands, gathered rows, expert bias, gpt-oss activation in mode 1); padding slots stay unwritten."""
    torch.manual_seed(5)
    dev = "cuda"
    C = ops.native()
    T, E, k, K, N = 400, 8, 4, 2944, 5760 if mode == 1 else 2880
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    xq, xs = ops._quant_groups_padded(x, K)
    wq, ws = ops.quant_fp8_block_weight(torch.randn(E, N, K, device=dev, dtype=torch.bfloat16) * 0.03)
    bias = torch.randn(E, N, device=dev, dtype=torch.bfloat16) * 0.1
    ids, _ = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    n = T * k
    max_p = ((n + E * (tile - 1)) + tile - 1) // tile * tile
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // tile, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sorted_ids, tile_e, offs, total, inv, tile)
    width = N // 2 if mode == 1 else N
    y = torch.full((max_p, width), 7.0, device=dev, dtype=torch.bfloat16)
    C.moe_gemm4_fp8(xq, xs, k, sorted_ids, tile_e, wq, ws, y, mode, 2, 1.702, 7.0, False, bias, tile, 8, total)
    torch.cuda.synchronize()
    xd = xq.float() * xs.repeat_interleave(128, 1)[:, :K]
    wd = ops.dequant_fp8_block_weight(wq, ws).float()
    sid = sorted_ids.long()
    live = sid >= 0
    te = tile_e.long().repeat_interleave(tile)[:max_p]
    ref = torch.zeros(max_p, N, device=dev)
    for e in range(E):
        rows = live & (te == e)
        if rows.any():
            ref[rows] = xd[sid[rows] // k] @ wd[e].T + bias[e].float()
    if mode == 1:
        g, u = ref[:, 0::2].clamp(max=7.0), ref[:, 1::2].clamp(-7.0, 7.0)
        ref = (u + 1) * g * torch.sigmoid(1.702 * g)
    got = y.float()
    m = ref[live].abs().max().item()
    assert (got[live] - ref[live]).abs().max().item() < 0.01 * m + 1e-2
    assert (got[~live] == 7.0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("T,E,k,d,F,act", [(700, 16, 4, 512, 2880, 2), (300, 8, 8, 256, 256, 0)])
def test_moe_fp8_fused_act_quant_gpu(T, E, k, d, F, act):
    """The 256-row first GEMM's fused epilogue quantisation (hq / hs) is bit
    for bit the unfused path: bf16 h from the same kernel, then
    quant_fp8_groups into K-padded rows (valid rows only; padding columns 0)."""
    torch.manual_seed(2)
    dev = "cuda"
    C = ops.native()
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1q, w1s = ops.quant_fp8_block_weight(torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.03)
    w1q = ops.pad_fp8_k(w1q, c128(d))
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    ids, _ = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    bm = C.moe_tile_m_prefill()
    n = T * k
    max_p = ((n + E * (bm - 1)) + bm - 1) // bm * bm
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // bm, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sorted_ids, tile_e, offs, total, inv, bm)
    xq, xs = ops._quant_groups_padded(x, c128(d))
    Kp2 = c128(F)
    h = torch.empty(max_p, F, dtype=torch.bfloat16, device=dev)
    C.moe_gemm_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, h, 1, act, 1.702, 7.0, False, b1, bm)
    ref_q, ref_s = ops._quant_groups_padded(h, Kp2)
    hq = torch.zeros(max_p, Kp2, dtype=ops.FP8, device=dev)
    hs = torch.zeros(max_p, Kp2 // 128, dtype=torch.float32, device=dev)
    C.moe_gemm_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, torch.empty(0, F, dtype=torch.bfloat16, device=dev),
                   1, act, 1.702, 7.0, False, b1, bm, hq, hs)
    valid = sorted_ids >= 0
    assert torch.equal(hs[valid], ref_s[valid])
    assert torch.equal(hq.view(torch.uint8)[valid], ref_q.view(torch.uint8)[valid])


def test_fused_norm_act_quant_cpu_matches_unfused():
    torch.manual_seed(0)
    x = torch.randn(6, 256).to(torch.bfloat16)
    res = torch.randn(6, 256).to(torch.bfloat16)
    w = (torch.rand(256) + 0.5).to(torch.bfloat16)
    r2 = res.clone()
    q, s = ops.rms_norm_quant(x, w, 1e-5, r2)
    xx, rr = x.clone(), res.clone()
    ops.fused_add_rms_norm(xx, rr, w, 1e-5)
    q2, s2 = ops.quant_fp8_rows(xx)
    assert torch.equal(r2, rr) and torch.allclose(s, s2) and torch.equal(q.float(), q2.float())
    h = torch.randn(6, 2 * 128).to(torch.bfloat16)
    qa, sa = ops.gated_act_quant(h, ops.ACT_SILU)
    qb, sb = ops.quant_fp8_rows(ops.gated_act(h, ops.ACT_SILU))
    assert torch.allclose(sa, sb) and torch.equal(qa.float(), qb.float())


@pytest.mark.gpu
@pytest.mark.parametrize("d", [256, 4096, 8192])
def test_fused_norm_act_quant_gpu(d):
    torch.manual_seed(1)
    x = torch.randn(37, d, device="cuda").to(torch.bfloat16)
    res = torch.randn(37, d, device="cuda").to(torch.bfloat16)
    w = (torch.rand(d, device="cuda") + 0.5).to(torch.bfloat16)
    for with_res in (False, True):
        r_gpu = res.clone() if with_res else None
        q, s = ops.rms_norm_quant(x, w, 1e-5, r_gpu)
        r_cpu = res.cpu().clone() if with_res else None
        qr, sr = ops.rms_norm_quant(x.cpu(), w.cpu(), 1e-5, r_cpu)
        if with_res:
            torch.testing.assert_close(r_gpu.cpu().float(), r_cpu.float(), atol=0, rtol=0)
        torch.testing.assert_close(s.cpu(), sr, rtol=2e-2, atol=1e-6)
        deq, deq_r = q.float().cpu() * s.cpu(), qr.float() * sr
        assert (deq - deq_r).abs().max() <= 0.07 * deq_r.abs().max()
    h = torch.randn(37, 2 * d, device="cuda").to(torch.bfloat16)
    for mode in (0, 2):
        qa, sa = ops.gated_act_quant(h, mode)
        qb, sb = ops.gated_act_quant(h.cpu(), mode)
        torch.testing.assert_close(sa.cpu(), sb, rtol=2e-2, atol=1e-6)
        deq, deq_r = qa.float().cpu() * sa.cpu(), qb.float() * sb
        assert (deq - deq_r).abs().max() <= 0.07 * deq_r.abs().max()


# ---------------------------------------------------------------- fp8 latent (MLA) cache
def test_engine_fp8_mla_kv_cpu():
    """DeepSeek (MLA) with an fp8 latent cache runs end to end (CPU reference ops)."""
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    outs = {}
    for kvd in ("auto", "fp8"):
        cfg = EngineConfig.create("tiny-deepseek", device="cpu", block_size=16, num_gpu_blocks=64,
                                  max_num_batched_tokens=256, max_num_seqs=4, max_model_len=512,
                                  kv_cache_dtype=kvd)
        eng = LLMEngine(cfg, capture_graphs=False)
        assert eng.runner.kv.dtype == (F8 if kvd == "fp8" else torch.bfloat16)
        reqs = eng.generate([list(range(3, 40)), [7] * 20], SamplingParams(max_tokens=6, temperature=0.0,
                                                                           ignore_eos=True))
        outs[kvd] = [r.output_token_ids for r in reqs]
    assert all(len(o) == 6 for o in outs["fp8"])
    assert [o[0] for o in outs["fp8"]] == [o[0] for o in outs["auto"]]


@pytest.mark.gpu
@pytest.mark.parametrize("H,bs,lens", [(128, 64, [1000, 4096, 7]), (128, 16, [1, 65, 300]),
                                       (64, 64, [777, 129]), (20, 16, [1, 63, 300])])
def test_mla_fp8_cache_kernels(H, bs, lens):
    """HIP rope+latent-cache write (fp8) and MLA attention (v2 for 64/128 heads,
    v1 otherwise) vs the fp32 reference over the same fp8 cache."""
    dev = "cuda"
    torch.manual_seed(3)
    ks = 0.5
    nb_per = max(math.ceil(L / bs) for L in lens)
    nb = len(lens) * nb_per + 3
    pool = torch.zeros(nb, 2, bs, 576, dtype=F8, device=dev)  # non-contiguous layer view
    cache = pool[:, 1]
    cache.copy_(ref.to_cache(torch.randn(nb, bs, 576, device=dev) * 2, F8, ks))
    bt = torch.stack([torch.randperm(nb, device=dev)[:nb_per] for _ in lens]).int()
    R = len(lens)
    q = torch.randn(R, H * 576, dtype=torch.bfloat16, device=dev)
    rows = torch.arange(R, dtype=torch.int32, device=dev)
    ln = torch.tensor(lens, dtype=torch.int32, device=dev)
    want = ref.mla_attention(q, cache, bt, rows, ln, H, 576 ** -0.5, ks)
    for split in (None, (64, math.ceil(max(lens) / 64))):
        got = ops.mla_attention(q, cache, bt, rows, ln, H, 576 ** -0.5, split=split, kv_scale=ks)
        _close(got, want)
    # rope + fp8 latent write: HIP vs reference on the same inputs
    T = 29
    qf = torch.randn(T, H * 192, dtype=torch.bfloat16, device=dev)
    kv = torch.randn(T, 576, dtype=torch.bfloat16, device=dev) * 3
    pos = torch.randint(0, 4000, (T,), device=dev)
    cs = ref.rope_cos_sin(64, 4096, 10000.0, device=dev)
    slots = torch.randperm(8 * bs, device=dev)[:T]
    slots[2] = -1
    ca = torch.zeros(8, bs, 576, dtype=F8, device=dev)
    cb = torch.zeros_like(ca)
    qa = torch.zeros(T, H * 576, dtype=torch.bfloat16, device=dev)
    qb = torch.zeros_like(qa)
    ops.mla_rope_cache(qf, qa, kv[:, :512], kv[:, 512:], pos, cs, H, slots, ca, kv_scale=ks)
    ref.mla_rope_cache(qf, qb, kv[:, :512], kv[:, 512:], pos, cs, H, slots, cb, ks)
    _close(qa, qb, atol=2e-2, rtol=2e-2)
    # fp8 codes may differ by one ulp where the bf16 -> fp32 rounding paths differ
    _close(ca.float() * ks, cb.float() * ks, atol=0.07 * ks, rtol=0.07)
