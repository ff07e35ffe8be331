"""Medium-M decode GEMM (csrc/ops/mgemm.hip) against an fp32 PyTorch
reference: M 33..128 (row clamping, partial token blocks), N not a multiple of
the tile (row clamping + dropped rows), K splits that do not divide the k-steps,
3- and 4-stage rings, split-K partials + reduce, hipGraph capture."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x, w):
    return (x.float() @ w.float().T)


@pytest.mark.parametrize("M", [33, 64, 80, 96, 128])
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


@pytest.mark.parametrize("M", [33, 64, 100, 128])
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
