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


@pytest.mark.parametrize("T,Hq,Hkv,D", [(1, 64, 8, 128), (37, 64, 8, 128), (5, 32, 4, 128), (9, 16, 2, 64),
                                        (3, 8, 8, 256), (130, 40, 8, 128)])
def test_qk_rms_norm_in_place(T, Hq, Hkv, D):
    """Qwen3 per-head q/k RMSNorm inside the fused QKV buffer: q and k heads
    match the fp32 reference, V is untouched."""
    torch.manual_seed(0)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16) * 3
    qw = torch.randn(D, device=DEV, dtype=torch.bfloat16)
    kw = torch.randn(D, device=DEV, dtype=torch.bfloat16)
    want = qkv.clone()
    q = ref.rms_norm(want[:, : Hq * D].reshape(-1, D), qw, 1e-6).view(T, -1)
    k = ref.rms_norm(want[:, Hq * D: (Hq + Hkv) * D].reshape(-1, D), kw, 1e-6).view(T, -1)
    got = qkv.clone()
    ops.qk_rms_norm(got, qw, kw, Hq, Hkv, 1e-6)
    _close(got[:, : Hq * D], q)
    _close(got[:, Hq * D: (Hq + Hkv) * D], k)
    assert torch.equal(got[:, (Hq + Hkv) * D:], qkv[:, (Hq + Hkv) * D:])


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
    # device-side split size (hipGraph replay): the grid's 8 splits re-sized to 640 keys
    o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, split=(16384, 8), max_ctx=max(lens),
                         split_dev=torch.tensor([640], dtype=torch.int32, device=DEV))
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


@pytest.mark.parametrize("Hq,Hkv,D,bs,groups,fp8,variant", [
    (64, 8, 128, 64, [(2048, 2), (1024, 3), (512, 4), (0, 3)], False, 2),   # 2 passes (4 members at G=8)
    (64, 8, 128, 64, [(3072, 2), (1024, 2)], False, 1),                        # 1 pass
    (32, 8, 128, 16, [(640, 7), (320, 2)], False, 2),                          # G 4: up to 8 members
    (64, 8, 64, 64, [(1024, 3), (768, 2)], False, 1),
    (16, 1, 128, 64, [(1536, 2), (512, 2)], False, 2),                         # G 16: one member per pass
    (64, 8, 128, 64, [(2048, 3), (1024, 2)], True, 2),
    (64, 8, 128, 64, [(2048, 17), (1088, 5), (512, 2), (0, 2)], False, 3),    # LDS-DMA: 16 members, partial tile
    (32, 8, 128, 128, [(1536, 33), (640, 3)], False, 3),                       # G 4: 32 members
    (64, 8, 64, 64, [(1024, 9), (704, 4)], False, 3),
    (64, 8, 128, 16, [(1040, 5), (2048, 12)], False, 3),                      # 16-key blocks, partial tile
    (64, 8, 64, 32, [(608, 3), (1024, 2)], False, 3),
])
def test_paged_decode_shared_prefix(Hq, Hkv, D, bs, groups, fp8, variant):
    """Shared-prefix (cascade) decode: prefixes read once per group by the
    prefix kernel, suffixes by the per-sequence kernel, merged by the reduce
    kernel - against the fp32 reference and the plain kernel; with sinks."""
    from shared_prefix_util import shared_tables

    torch.manual_seed(4)
    bt_np, lens_np, nb = shared_tables(groups, [1, 63, 64, 65, 300, 7], bs, seed=2)
    kc, vc = _cache(nb + 2, Hkv, bs, D, L=2)
    kc.normal_()
    vc.normal_()
    if fp8:
        kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
    B = len(lens_np)
    bt = torch.from_numpy(bt_np).to(DEV)
    sl = torch.from_numpy(lens_np).to(DEV)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    sinks = torch.randn(Hq, device=DEV)
    scale = D ** -0.5
    plan = ops.shared_prefix_plan(bt_np, lens_np, bs, G=Hq // Hkv, Hkv=Hkv, variant=variant, min_prefix=256,
                                  min_chunk=256)
    assert plan is not None and plan.items >= 2 and plan.np == variant
    casc = ops.cascade_tensors(plan, DEV)
    for sk in (None, sinks):
        r = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, 0, sk)
        suffix = int((lens_np - plan.sstart).max())
        for split in [None, (64, -(-suffix // 64)), (4096, 2)]:
            if split is None:
                split = ops.decode_split_plan(suffix, B, Hkv, Hq // Hkv)
            o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, 0, sk, split=split, cascade=casc)
            _close(o, r)
        plain = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, 0, sk, max_ctx=int(lens_np.max()))
        _close(o, plain)



@pytest.mark.parametrize("M,plan", [(m, p) for m in (33, 64, 100, 128)
                                    for p in ((1, 1, 3), (2, 3, 3), (4, 2, 3), (2, 5, 4))] +
                         [(m, p) for m in (150, 256) for p in ((1, 1, 3), (1, 4, 4), (2, 3, 3))])
def test_mgemm_fp8(M, plan):
    """fp8 W8A8 medium-M GEMM (per-token x per-channel scales) vs the fp32 reference
    of the dequantised operands, and against hipBLASLt's scaled GEMM."""
    torch.manual_seed(7)
    N, K = 1280, 1024
    F8 = torch.float8_e4m3fn
    xq = torch.randn(M, K, device=DEV).to(F8)
    wq = (torch.randn(N, K, device=DEV) * 0.5).to(F8)
    xs = torch.rand(M, 1, device=DEV) * 0.02 + 0.001
    ws = torch.rand(1, N, device=DEV) * 0.02 + 0.001
    want = (xq.float() * xs) @ (wq.float() * ws.view(-1, 1)).t()
    got = ops.mgemm_fp8(xq, xs, wq, ws, plan)
    _close(got, want, atol=2e-3, rtol=2e-2)
    lib = torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16)
    _close(got, lib, atol=2e-3, rtol=2e-2)


@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (77, 512, 1024), (256, 768, 128), (1000, 1280, 2048),
                                   (4608, 1024, 8192), (300, 512, 8192), (4608, 8192, 8192)])
@pytest.mark.parametrize("variant", [0, 1, 3, 6])
def test_pgemm(M, N, K, variant):
    """Prefill GEMM (256 x 256 LDS-DMA tiles, counted-vmcnt pipeline) vs the fp32
    reference; K = 64 and 128 exercise the prologue / tail waits without a steady state;
    odd M the clamped rows. Fused SiLU-and-mul epilogue on the interleaved gate/up layout.
    Both variants with and without the split-K tail: (1000, 1280, 2048) = 20 tiles in 4 splits,
    (300, 512, 8192) = tail only (16 splits), (4608, 8192, 8192) = 512 data-parallel tiles +
    64 tail tiles in 4 splits (the 70B o-projection at a 4608-token step)."""
    torch.manual_seed(11)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=DEV) * 2 - 1) * 0.05).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    _close(ops.pgemm(x, w, variant=variant), ref, atol=2e-2, rtol=2e-2)
    _close(ops.pgemm(x, w, variant=variant, split_k=False), ref, atol=2e-2, rtol=2e-2)
    g, u = ref[:, : N // 2], ref[:, N // 2:]
    if variant != 6:  # the persistent variant has no packed-layout (epi 1) form
        _close(ops.pgemm(x, ops.pgemm_pack_gate_up(w), epi=1, variant=variant), g * torch.sigmoid(g) * u,
               atol=2e-2, rtol=3e-2)
    if variant in (3, 6):  # fused SiLU on the plain [gate; up] weight (the engine's layout)
        _close(ops.pgemm_silu(x, w, variant=variant), g * torch.sigmoid(g) * u, atol=2e-2, rtol=3e-2)


@pytest.mark.parametrize("variant", [3, 4, 5, 6])
def test_pgemm_v3_schedules_and_silu_std(variant):
    """Variants 3-5 (4 waves x 128 x 128, the whole K-step register-resident, LDS-DMA two steps
    ahead) at a 70B-like prefill shape with an odd M, split-K tail on and off, and the fused
    SiLU on the plain [gate; up] weight (F = 1408: 11 tiles of 128) vs the fp32 reference."""
    torch.manual_seed(12)
    M, K = 1030, 4096
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(2816, K, device=DEV) * 2 - 1) * 0.05).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    _close(ops.pgemm(x, w, variant=variant), ref, atol=2e-2, rtol=2e-2)
    _close(ops.pgemm(x, w, variant=variant, split_k=False), ref, atol=2e-2, rtol=2e-2)
    g, u = ref[:, :1408], ref[:, 1408:]
    _close(ops.pgemm_silu(x, w, variant=variant), g * torch.sigmoid(g) * u, atol=2e-2, rtol=3e-2)


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


@pytest.mark.parametrize("D,bs", [(64, 16), (64, 64), (128, 64)])
def test_paged_prefill_window_sinks(D, bs):
    Hq, Hkv = 64, 8
    shapes = [(300, 300), (77, 500)]
    ctx = [c for _, c in shapes]
    kc, vc, bt = _paged_setup(ctx, Hkv, D, bs, seed=6)
    ql = [a for a, _ in shapes]
    qs = [0, ql[0]]
    q = torch.randn(sum(ql), Hq * D, device=DEV, dtype=torch.bfloat16)
    sinks = torch.randn(Hq, device=DEV)
    args = [torch.tensor(x, dtype=torch.int32, device=DEV) for x in (qs, ql, ctx)]
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, D ** -0.5, 128, sinks)
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, D ** -0.5, 128, sinks)
    _close(o, r)


def test_sample_greedy_and_logprob():
    torch.manual_seed(7)
    logits = torch.randn(9, 128256, device=DEV).to(torch.bfloat16)
    ids, lp = ops.sample(logits, want_logprob=True)
    assert torch.equal(ids, logits.float().argmax(-1))
    ref_lp = torch.log_softmax(logits.float(), -1).gather(-1, ids[:, None]).squeeze(-1)
    _close(lp, ref_lp, atol=1e-3, rtol=1e-3)


def test_sample_split_rows_match_unsplit():
    """Small batches split each row over several workgroups: the seeded Gumbel pick and
    the log-prob equal those of the same rows inside a batch large enough to run unsplit."""
    torch.manual_seed(9)
    V = 151936
    big = torch.randn(600, V, device=DEV).to(torch.bfloat16)
    temps = torch.full((600,), 0.8, device=DEV)
    seeds = torch.arange(600, device=DEV, dtype=torch.int64) * 31 + 5
    ids_big, lp_big = ops.sample(big, temps, seeds, want_logprob=True)
    ids_small, lp_small = ops.sample(big[:5].contiguous(), temps[:5], seeds[:5], want_logprob=True)
    assert torch.equal(ids_small, ids_big[:5])
    _close(lp_small, lp_big[:5], atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("B", [4, 600])   # split rows (small batch) and unsplit
def test_sample_logprob_masked_rows(B):
    """Rows with -inf entries (top-k / top-p / min_p masks): the log-prob of the
    pick must be finite and match the masked log-softmax (a thread whose first
    entries are masked used to turn its partial sum-exp into NaN)."""
    torch.manual_seed(10)
    V = 128256
    x = torch.randn(B, V, device=DEV)
    topk = torch.full((B,), 40, dtype=torch.int32, device=DEV)
    temps = torch.full((B,), 0.9, device=DEV)
    m = ops.topk_topp_mask(x.clone(), topk, None, temps)
    m[1::2, ::3] = float("-inf")                       # and a min_p-like strided mask on odd rows
    m[1::2, x.argmax(-1)[1]] = 5.0                     # keep one finite entry in those rows
    seeds = torch.arange(B, device=DEV, dtype=torch.int64) * 13 + 1
    for t in (None, temps):
        ids, lp = ops.sample(m, t, seeds if t is not None else None, want_logprob=True)
        assert torch.isfinite(lp).all()
        assert torch.isfinite(m.gather(1, ids[:, None])).all()       # never picks a masked entry
        want = torch.log_softmax(m, -1).gather(1, ids[:, None]).squeeze(1)
        _close(lp, want, atol=1e-3, rtol=1e-3)


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


@pytest.mark.parametrize("engine", [0, 1])   # register-staged, LDS-staged (LDS-DMA)
def test_kvx_copy_blocks_and_reslice(engine):
    C = ops.native()
    L, H, bs, D = 3, 8, 16, 128
    src = torch.randn(10, L, 2, H, bs, D, device=DEV).to(torch.bfloat16)
    dst = torch.zeros(12, L, 2, H, bs, D, device=DEV, dtype=torch.bfloat16)
    bb = src[0].numel() * 2
    pairs = torch.tensor([[1, 5], [7, 0], [3, 11]], dtype=torch.int32, device=DEV)
    segs = torch.tensor([[0, 0, bb]], dtype=torch.int64, device=DEV)
    C.kvx_copy_blocks(dst, src.data_ptr(), bb, bb, pairs, segs, bb, engine)
    torch.cuda.synchronize()
    for s_, d_ in [(1, 5), (7, 0), (3, 11)]:
        assert torch.equal(dst[d_], src[s_])
    # TP re-slice: decoder rank 1 of 4 takes heads [2, 4)
    hl = 2
    dst2 = torch.zeros(4, L, 2, hl, bs, D, device=DEV, dtype=torch.bfloat16)
    head = bs * D * 2
    sg = [(((l * 2 + kv) * H + 2) * head, ((l * 2 + kv) * hl) * head, hl * head) for l in range(L) for kv in range(2)]
    C.kvx_copy_blocks(dst2, src.data_ptr(), dst2[0].numel() * 2, bb,
                      torch.tensor([[4, 2]], dtype=torch.int32, device=DEV),
                      torch.tensor(sg, dtype=torch.int64, device=DEV), hl * head, engine)
    torch.cuda.synchronize()
    assert torch.equal(dst2[2], src[4][:, :, 2:4])
    # SDMA path
    dst3 = torch.zeros_like(dst)
    C.kvx_dma_blocks(dst3, src.data_ptr(), bb, bb, torch.tensor([[2, 3], [3, 4], [9, 1]], dtype=torch.int32), bb)
    torch.cuda.synchronize()
    assert torch.equal(dst3[3], src[2]) and torch.equal(dst3[4], src[3]) and torch.equal(dst3[1], src[9])


@pytest.mark.parametrize("E,k,scoring,ng,tg,renorm", [(128, 4, 2, 1, 1, False), (32, 4, 2, 1, 1, False),
                                                       (256, 8, 1, 8, 4, True), (64, 6, 0, 1, 1, False)])
def test_moe_topk(E, k, scoring, ng, tg, renorm):
    torch.manual_seed(9)
    T = 37
    logits = torch.randn(T, E, device=DEV)
    bias = torch.randn(E, device=DEV) * 0.1 if scoring == 1 else None
    ids, w = ops.moe_topk(logits, k, scoring, bias, ng, tg, renorm, 2.5 if scoring == 1 else 1.0)
    rid, rw = ref.moe_topk(logits, k, scoring, bias, ng, tg, renorm, 2.5 if scoring == 1 else 1.0)
    # same expert sets (order may differ only on exact ties)
    assert torch.equal(torch.sort(ids.long(), -1).values, torch.sort(rid.long(), -1).values)
    po = torch.sort(ids.long(), -1).indices
    pr = torch.sort(rid.long(), -1).indices
    _close(w.gather(-1, po), rw.gather(-1, pr), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("T,E,k,d,F,act", [(1, 8, 2, 256, 128, 2), (37, 32, 4, 2880, 2880, 2),
                                            (19, 128, 4, 512, 256, 2), (64, 16, 2, 1024, 512, 0),
                                            # prefill-sized: 256-row tiles of the bf16 v3 kernel (>= 96 rows
                                            # per expert), experts spanning several tiles, gpt-oss widths
                                            (1024, 8, 2, 1024, 512, 0), (800, 16, 4, 2880, 2880, 2)])
def test_moe_experts(T, E, k, d, F, act):
    torch.manual_seed(10)
    x = torch.randn(T, d, device=DEV, dtype=torch.bfloat16)
    w1 = (torch.randn(E, 2 * F, d, device=DEV) * d ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(E, d, F, device=DEV) * F ** -0.5).to(torch.bfloat16)
    b1 = (torch.randn(E, 2 * F, device=DEV) * 0.1).to(torch.bfloat16)
    b2 = (torch.randn(E, d, device=DEV) * 0.1).to(torch.bfloat16)
    logits = torch.randn(T, E, device=DEV)
    ids, w = ops.moe_topk(logits, k, 2)
    o = ops.moe_experts(x, ids, w, w1, w2, act, b1=b1, b2=b2)
    r = ref.moe_forward(x, ids, w, w1, w2, act, b1=b1, b2=b2)
    _close(o, r, atol=3e-2, rtol=3e-2)
    # EP-style masking: experts outside the local range are ignored
    ids2 = ids.clone()
    ids2[ids2 >= E // 2] = -1
    o2 = ops.moe_experts(x, ids2, w, w1, w2, act, b1=b1, b2=b2)
    r2 = ref.moe_forward(x, ids2, w, w1, w2, act, b1=b1, b2=b2)
    _close(o2, r2, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("v8", [False, True])
@pytest.mark.parametrize("tile", ["256", "192"])
@pytest.mark.parametrize("T,E,k,d,F,act", [(1024, 8, 2, 1024, 512, 0), (800, 16, 4, 2880, 2880, 2),
                                            (2048, 32, 8, 1024, 768, 0)])
def test_moe_experts_bf16_v4(T, E, k, d, F, act, tile, v8, monkeypatch):
    """The v4 bf16 grouped GEMM (csrc/ops/moe4.hip: 4-wave PGR2 tiles of 256 or 192 rows, A rows
    gathered by the LDS-DMA, gated activation in registers) and its persistent form (v8,
    csrc/ops/moe8.hip) vs the fp32 reference, with biases, gpt-oss widths (N = 5760 and 2880:
    partial last column tiles) and EP-style masked experts."""
    monkeypatch.setattr(ops, "MOE_BF16_V4", True)
    monkeypatch.setattr(ops, "MOE_BF16_V8", v8)
    monkeypatch.setattr(ops, "MOE4_TILE", tile)
    torch.manual_seed(13)
    x = torch.randn(T, d, device=DEV, dtype=torch.bfloat16)
    w1 = (torch.randn(E, 2 * F, d, device=DEV) * d ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(E, d, F, device=DEV) * F ** -0.5).to(torch.bfloat16)
    b1 = (torch.randn(E, 2 * F, device=DEV) * 0.1).to(torch.bfloat16)
    b2 = (torch.randn(E, d, device=DEV) * 0.1).to(torch.bfloat16)
    ids, w = ops.moe_topk(torch.randn(T, E, device=DEV), k, 2)
    _close(ops.moe_experts(x, ids, w, w1, w2, act, b1=b1, b2=b2),
           ref.moe_forward(x, ids, w, w1, w2, act, b1=b1, b2=b2), atol=3e-2, rtol=3e-2)
    ids2 = ids.clone()
    ids2[ids2 >= E // 2] = -1
    _close(ops.moe_experts(x, ids2, w, w1, w2, act), ref.moe_forward(x, ids2, w, w1, w2, act),
           atol=3e-2, rtol=3e-2)
