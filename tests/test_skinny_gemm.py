"""Skinny decode GEMM (csrc/ops/skinny_gemm.hip) vs an fp32 reference, across
M buckets, split-K factors and ragged N."""
import pytest
import torch

from llmd_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 3, 16, 17, 33, 64])
@pytest.mark.parametrize("N,K", [(1000, 256), (4096, 1024), (10240, 8192)])
def test_skinny_gemm_matches_fp32(M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    want = (x.float() @ w.float().T)
    for ns in (1, 3, ops.skinny_splits(M, N, K)):
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        part = torch.empty(max(1, ns) * M * N, dtype=torch.float32, device="cuda")
        ops.native().skinny_gemm(y, x, w, ns, part)
        err = (y.float() - want).abs().max().item()
        tol = 2e-2 * max(1.0, want.abs().max().item())
        assert err < tol, (M, N, K, ns, err)
    y2 = ops.linear(x, w)
    assert (y2.float() - want).abs().max().item() < 2e-2 * max(1.0, want.abs().max().item())


def test_linear_strided_rows_and_bias():
    x = torch.randn(8, 640, device="cuda").bfloat16()[:, :512]   # row stride 640
    w = torch.randn(300, 512, device="cuda").bfloat16()
    b = torch.randn(300, device="cuda").bfloat16()
    want = x.float() @ w.float().T + b.float()
    got = ops.linear(x, w, b)
    assert (got.float() - want).abs().max().item() < 2e-2 * want.abs().max().item()
