"""fp8 W8A8 prefill GEMM (csrc/ops/pgemm8.hip) vs the fp32 PyTorch oracle of the
same op: y = (xs . xq) (ws . wq)^T with per-token / per-channel scales, and the
fused silu(gate) * up epilogue on the plain [gate; up] weight. Shapes cover a
partial last row tile, odd K-step counts (the 2-step unroll's tail), a single
K-step, and the engine dispatch in ops.fp8_linear."""
import pytest
import torch

from llmd_amd import ops

pytestmark = pytest.mark.gpu


def _q(shape, gen, scale=1.0):
    x = torch.randn(shape, generator=gen, device="cuda") * scale
    return ops.quant_fp8_rows(x.to(torch.bfloat16))


def _ref(xq, xs, wq, ws):
    return (xq.float() * xs.view(-1, 1)) @ (wq.float() * ws.view(-1, 1)).t()


@pytest.mark.parametrize("M,N,K", [(1, 256, 128), (300, 512, 384), (513, 768, 1024), (1030, 1280, 640),
                                   (256, 256, 256)])
def test_pgemm_fp8_matches_fp32(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    xq, xs = _q((M, K), g)
    wq, ws = ops.quant_fp8_weight(torch.randn(N, K, generator=g, device="cuda") * 0.05)
    y = ops.pgemm_fp8(xq, xs, wq, ws)
    r = _ref(xq, xs, wq, ws)
    torch.cuda.synchronize()
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    err = (y.float() - r).abs().max().item()
    assert err <= 1e-2 * r.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("M,F,K", [(300, 128, 256), (777, 384, 512)])
def test_pgemm_fp8_silu_epilogue(M, F, K):
    g = torch.Generator(device="cuda").manual_seed(7 * M + F)
    xq, xs = _q((M, K), g)
    wq, ws = ops.quant_fp8_weight(torch.randn(2 * F, K, generator=g, device="cuda") * 0.05)
    y = ops.pgemm_fp8(xq, xs, wq, ws, epi=3)
    h = _ref(xq, xs, wq, ws)
    r = torch.nn.functional.silu(h[:, :F]) * h[:, F:]
    torch.cuda.synchronize()
    assert y.shape == (M, F)
    err = (y.float() - r).abs().max().item()
    assert err <= 2e-2 * r.abs().max().item() + 1e-3, err


def test_pgemm_fp8_exact_integers():
    """Small integers are exact in e4m3 and in the fp32 accumulator: any
    fragment-layout error shows as a wrong element, not as noise."""
    g = torch.Generator(device="cuda").manual_seed(3)
    M, N, K = 260, 512, 384
    x = torch.randint(-3, 4, (M, K), generator=g, device="cuda").float()
    w = torch.randint(-3, 4, (N, K), generator=g, device="cuda").float()
    xq, wq = x.to(torch.float8_e4m3fn), w.to(torch.float8_e4m3fn)
    one_m = torch.ones(M, 1, device="cuda")
    one_n = torch.ones(1, N, device="cuda")
    y = ops.pgemm_fp8(xq, one_m, wq, one_n)
    r = x @ w.t()
    torch.cuda.synchronize()
    # |r| <= 9 * 384 = 3456: exact in bf16 only up to 256, so compare after rounding r to bf16
    assert torch.equal(y.float(), r.to(torch.bfloat16).float())


@pytest.mark.parametrize("M,N,K", [(300, 512, 2048), (513, 256, 4096)])
def test_pgemm_fp8_split_k_tail(M, N, K):
    """A last wave at most half full runs split over K (fp32 partials + reduce): same result."""
    g = torch.Generator(device="cuda").manual_seed(K)
    xq, xs = _q((M, K), g)
    wq, ws = ops.quant_fp8_weight(torch.randn(N, K, generator=g, device="cuda") * 0.05)
    y0 = ops.pgemm_fp8(xq, xs, wq, ws, split_k=False)
    y1 = ops.pgemm_fp8(xq, xs, wq, ws, split_k=True)
    r = _ref(xq, xs, wq, ws)
    torch.cuda.synchronize()
    for y in (y0, y1):
        err = (y.float() - r).abs().max().item()
        assert err <= 1e-2 * r.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("M,N,K", [(1030, 16384, 256), (300, 1024, 2048), (2100, 8192, 512)])
def test_pgemm_fp8_persistent(M, N, K):
    """Persistent form: tiles walked as one K-step stream per workgroup (more tiles than
    workgroups in the first and last shapes), epilogue from the accumulators with the
    LDS-staged scales; same result as the oracle."""
    g = torch.Generator(device="cuda").manual_seed(N + K)
    xq, xs = _q((M, K), g)
    wq, ws = ops.quant_fp8_weight(torch.randn(N, K, generator=g, device="cuda") * 0.05)
    y = ops.pgemm_fp8(xq, xs, wq, ws, persistent=True)
    r = _ref(xq, xs, wq, ws)
    torch.cuda.synchronize()
    err = (y.float() - r).abs().max().item()
    assert err <= 1e-2 * r.abs().max().item() + 1e-3, err
