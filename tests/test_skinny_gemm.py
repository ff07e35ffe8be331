"""Decode GEMM (csrc/ops/skinny_gemm.hip) vs an fp32 reference, across M
buckets, row-block / split-K / occupancy plans and ragged N."""
import pytest
import torch

from llmd_amd import ops

pytestmark = pytest.mark.gpu


def _check(y, want):
    err = (y.float() - want).abs().max().item()
    return err < 2e-2 * max(1.0, want.abs().max().item()), err


@pytest.mark.parametrize("M", [1, 3, 16, 17, 33, 64])
@pytest.mark.parametrize("N,K", [(1000, 256), (4096, 1024), (10240, 8192)])
def test_skinny_gemm_matches_fp32(M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    want = x.float() @ w.float().T
    plans = {ops.skinny_plan(M, N, K)}
    for rb in (1, 3, 4, 7, 8):
        for occ in (1, 2):
            if ops.native().skinny_supported(M, rb, occ):
                plans.add((rb, 1, occ))
                plans.add((rb, 3, occ))
    for plan in sorted(plans):
        ok, err = _check(ops.skinny_gemm(x, w, plan), want)
        assert ok, (M, N, K, plan, err)


def test_skinny_strided_rows_and_linear_bias(monkeypatch):
    monkeypatch.setattr(ops, "_SKINNY", True)
    x = torch.randn(8, 640, device="cuda").bfloat16()[:, :512]   # row stride 640
    w = torch.randn(300, 512, device="cuda").bfloat16()
    b = torch.randn(300, device="cuda").bfloat16()
    want = x.float() @ w.float().T + b.float()
    assert ops.skinny_ok(x, w)
    got = ops.linear(x, w, b)
    assert (got.float() - want).abs().max().item() < 2e-2 * want.abs().max().item()


def test_skinny_graph_capture():
    """The decode GEMM (and its split-K partials) replay inside a hipGraph."""
    x = torch.randn(32, 4096, device="cuda").bfloat16()
    w = (torch.randn(8192, 4096, device="cuda") * 0.02).bfloat16()
    plan = (4, 4, 2)
    ops.skinny_gemm(x, w, plan)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = ops.skinny_gemm(x, w, plan)
    x.copy_(torch.randn_like(x))
    g.replay()
    torch.cuda.synchronize()
    ok, err = _check(y, x.float() @ w.float().T)
    assert ok, err
