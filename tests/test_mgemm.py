"""Medium-M decode GEMM (csrc/ops/mgemm.hip) against an fp32 PyTorch
reference: M 33..256 (row clamping, partial token blocks), N not a multiple of
the tile (row clamping + dropped rows), K splits that do not divide the k-steps,
3- and 4-stage rings, split-K partials + reduce, hipGraph capture."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x, w):
    return (x.float() @ w.float().T)


@pytest.mark.parametrize("M", [33, 64, 80, 96, 128, 160, 192, 200, 256])
@pytest.mark.parametrize("N,K", [(640, 1024), (1028, 4160), (8192, 512)])
def test_mgemm_matches_fp32(M, N, K):
    from llmd_amd import ops

    torch.manual_seed(M * 7 + N)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    want = _ref(x, w)
    tol = 2e-2 * max(1.0, want.abs().max().item())
    for wrb in (1, 2, 4):
        for ns in (1, 3, 7):
            if ns > K // 64:
                continue
            for stages in (3, 4):
                if not ops.native().mgemm_lds(M, wrb, stages):
                    continue
                y = ops.mgemm(x, w, (wrb, ns, stages))
                err = (y.float() - want).abs().max().item()
                assert err <= tol, (M, N, K, wrb, ns, stages, err)


def test_mgemm_strided_x_and_linear_dispatch():
    from llmd_amd import ops

    x_big = torch.randn(96, 2048 + 64, device="cuda").bfloat16()
    x = x_big[:, :2048]  # row stride 2112 (multiple of 8)
    w = (torch.randn(1536, 2048, device="cuda") * 0.05).bfloat16()
    y = ops.mgemm(x, w, (2, 4, 4))
    assert (y.float() - _ref(x, w)).abs().max().item() <= 2e-2 * max(1.0, _ref(x, w).abs().max().item())
    # linear() falls back to hipBLASLt for shapes the table does not list
    assert torch.allclose(ops.linear(x.contiguous(), w).float(), _ref(x, w), atol=0.5, rtol=0.05)


def test_mgemm_graph_capture():
    from llmd_amd import ops

    x = torch.randn(128, 4096, device="cuda").bfloat16()
    w = (torch.randn(2048, 4096, device="cuda") * 0.05).bfloat16()
    plan = (2, 4, 4)
    ops.mgemm(x, w, plan)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = ops.mgemm(x, w, plan)
    for _ in range(2):
        x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        want = _ref(x, w)
        assert (y.float() - want).abs().max().item() <= 2e-2 * max(1.0, want.abs().max().item())


def test_mgemm_split_fixup_many_launches_two_streams():
    """The in-kernel split-K fixup (LLMD_MGEMM_FIXUP=1; per-tile counters on round-robin slabs, left
    zeroed by each launch; column-tile counts that are multiples of 8): > 256 back-to-back launches
    (every slab reused) interleaved on two streams at once, split counts that leave the last split
    short. Without the switch the same calls run the reduce kernel."""
    from llmd_amd import ops

    torch.manual_seed(5)
    ws = [(torch.randn(2048, 2560, device="cuda") * 0.05).bfloat16() for _ in range(2)]  # 16 column tiles
    xs = [torch.randn(64, 2560, device="cuda").bfloat16() for _ in range(6)]
    want = [[_ref(x, w) for w in ws] for x in xs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    torch.cuda.synchronize()
    for i in range(300):
        s = streams[i % 2]
        with torch.cuda.stream(s):
            outs.append((i % 6, i % 2, ops.mgemm(xs[i % 6], ws[i % 2], (2, 3 + i % 5, 3))))
    torch.cuda.synchronize()
    for xi, wi, y in outs:
        ref = want[xi][wi]
        assert (y.float() - ref).abs().max().item() <= 2e-2 * max(1.0, ref.abs().max().item()), (xi, wi)


@pytest.mark.parametrize("M", [33, 64, 100, 128, 176, 256])
@pytest.mark.parametrize("F,K", [(1536, 1024), (2004, 2048)])
def test_mgemm_silu_matches_fp32(M, F, K):
    """The ACT form (SiLU-and-mul in the epilogue on the plain [gate; up] weight) vs fp32:
    every wrb / stage ring it instantiates, F not a multiple of the tile's half (dropped rows)."""
    from llmd_amd import ops

    torch.manual_seed(M + F)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(2 * F, K, device="cuda") * 0.05).bfloat16()
    h = _ref(x, w)
    want = torch.nn.functional.silu(h[:, :F]) * h[:, F:]
    tol = 2e-2 * max(1.0, want.abs().max().item())
    for wrb in (2, 4):
        for stages in (3, 4):
            if not ops.native().mgemm_lds(M, wrb, stages):
                continue
            y = ops.mgemm_silu(x, w, (wrb, 1, stages))
            assert y.shape == (M, F)
            err = (y.float() - want).abs().max().item()
            assert err <= tol, (M, F, K, wrb, stages, err)


@pytest.mark.parametrize("M", [33, 64, 128])
@pytest.mark.parametrize("N,K,plan", [(8192, 8192, (1, 2, 4)), (8192, 28672, (4, 6, 3)), (1032, 1024, (2, 3, 3))])
def test_mgemm_add_rmsnorm_bit_identical(M, N, K, plan):
    """The o / down projection with the residual-add + RMSNorm in its split-K reduce
    (ops.mgemm_add_rmsnorm) against the two-kernel path it replaces (mgemm + fused_add_rms_norm):
    bit-identical output AND residual, and close to an fp32 reference; N not a multiple of 2048
    (partial per-thread chunks), the 70B o / down shapes and plans."""
    from llmd_amd import ops

    if not ops.native().mgemm_lds(M, plan[0], plan[2]):
        pytest.skip("no ring for this M")
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    res0 = torch.randn(M, N, device="cuda").bfloat16()
    g = (1 + 0.1 * torch.randn(N, device="cuda")).bfloat16()
    eps = 1e-5
    # two-kernel path
    y = ops.mgemm(x, w, plan)
    r_ref = res0.clone()
    ops.fused_add_rms_norm(y, r_ref, g, eps)
    # fused
    r = res0.clone()
    out = ops.mgemm_add_rmsnorm(x, w, plan, r, g, eps)
    torch.cuda.synchronize()
    assert torch.equal(r, r_ref)
    assert torch.equal(out, y)
    # and against fp32
    h = res0.float() + _ref(x, w)
    want = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * g.float()
    assert (out.float() - want).abs().max().item() < 5e-2 * max(1.0, want.abs().max().item())


def test_llama_decode_norm_fusion_greedy_equal(monkeypatch):
    """small-llama (40 sequences: decode M = 40, hipGraphs) decodes the same greedy tokens with
    the decode-GEMM reduce fusions (o / down + RMSNorm, QKV + RoPE + cache write) on and off. Its
    shapes are not in the shipped medium-M table, so a split-K plan is supplied for them in both
    runs; the fused reduces are bit-identical, so the logits and tokens are too."""
    from llmd_amd import ops
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    base = ops.mgemm_choice
    monkeypatch.setattr(ops, "mgemm_choice", lambda M, N, K: (1, 2, 3) if N in (1024, 1536) else base(M, N, K))
    calls = []
    fused, fused_rope = ops.mgemm_add_rmsnorm, ops.reduce_rope_cache
    monkeypatch.setattr(ops, "mgemm_add_rmsnorm", lambda *a, **k: calls.append(1) or fused(*a, **k))
    monkeypatch.setattr(ops, "reduce_rope_cache", lambda *a, **k: calls.append(2) or fused_rope(*a, **k))
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    prompts = [[(7 * i + j) % 1000 + 5 for j in range(40 + i)] for i in range(40)]

    def run():
        cfg = EngineConfig.create("small-llama", device="cuda", block_size=64, num_gpu_blocks=256,
                                  max_num_batched_tokens=4096, max_num_seqs=40, max_model_len=1024,
                                  cuda_graph_max_bs=64)
        return [r.output_token_ids for r in LLMEngine(cfg).generate(prompts, sp)]

    on = run()
    assert 1 in calls and 2 in calls, "the fused o / down / QKV paths never ran"
    monkeypatch.setattr(ops, "MGEMM_NORM", False)
    calls.clear()
    off = run()
    assert not calls
    assert on == off and all(len(t) == 6 for t in on)


@pytest.mark.parametrize("neox,fp8", [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize("M,Hq,Hkv,K,plan", [(64, 64, 8, 8192, (2, 3, 3)), (40, 8, 2, 1024, (1, 2, 3)),
                                             (128, 32, 4, 8192, (2, 6, 3))])  # 70B TP1 / small / 70B TP2 shard
def test_reduce_rope_cache_bit_identical(M, Hq, Hkv, K, plan, neox, fp8):
    """The decode QKV projection's split-K reduce fused with RoPE + the paged cache write
    (ops.mgemm_partials + ops.reduce_rope_cache) against mgemm + rope_cache: the same qkv rows
    (Q rotated, K / V as projected) and the same K / V cache bytes; padded rows (slot -1) skipped."""
    from llmd_amd import ops

    D, bs = 128, 64
    W = (Hq + 2 * Hkv) * D
    if not ops.native().mgemm_lds(M, plan[0], plan[2]):
        pytest.skip("no ring for this M")
    torch.manual_seed(M + Hq + K + int(neox) + 2 * int(fp8))
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(W, K, device="cuda") * 0.02).bfloat16()
    pos = torch.randint(0, 4000, (M,), device="cuda", dtype=torch.int64)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device="cuda").float() / D))
    ang = torch.arange(4096, device="cuda").float()[:, None] * inv[None]
    cos_sin = torch.cat([ang.cos(), ang.sin()], 1).contiguous()
    nblk = 64
    slots = torch.randperm(nblk * bs, device="cuda")[:M].to(torch.int64)
    slots[3] = -1
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    caches = [torch.zeros(nblk, Hkv, bs, D, device="cuda").to(dt) for _ in range(4)]
    ks, vs = (0.5, 0.25) if fp8 else (1.0, 1.0)
    # two-kernel path
    q1 = ops.mgemm(x, w, plan)
    ops.rope_cache(q1, pos, cos_sin, Hq, Hkv, D, slots, caches[0], caches[1], neox, ks, vs)
    # fused
    part, ns = ops.mgemm_partials(x, w, plan)
    q2 = torch.empty(M, W, device="cuda", dtype=torch.bfloat16)
    ops.reduce_rope_cache(part, ns, q2, pos, cos_sin, Hq, Hkv, D, slots, caches[2], caches[3], neox, ks, vs)
    torch.cuda.synchronize()
    assert torch.equal(q1, q2)
    assert torch.equal(caches[0].view(torch.uint8), caches[2].view(torch.uint8))
    assert torch.equal(caches[1].view(torch.uint8), caches[3].view(torch.uint8))
