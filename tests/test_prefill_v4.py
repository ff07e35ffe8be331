"""Prefill attention v4 (csrc/ops/attn_prefill.hip prefill_v4_kernel: 32x32x16 MFMAs, S^T's
accumulator as the PV operand, transposed V reads in its permuted key order) against the fp32
reference: fresh prompts, chunks over cached prefixes, blocks of 16 and 64 keys, GQA 8 / 4 / 1 /
2, sliding window + sinks, and the production ISL 5000 / 8192 shapes."""
import math

import pytest
import torch

from llmd_amd import ops
from llmd_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol=2e-2, rtol=2e-2):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=rtol)


def _paged(ctx, Hkv, D, bs, seed):
    torch.manual_seed(seed)
    nb = [(c + bs - 1) // bs for c in ctx]
    total = sum(nb) + 3
    kc = torch.randn(total, Hkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(total, Hkv, bs, D, device=DEV, dtype=torch.bfloat16)
    perm = torch.randperm(total)
    bt = torch.zeros(len(ctx), max(nb) + 1, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nb):
        bt[i, :n] = perm[o:o + n].int()
        o += n
    return kc, vc, bt.to(DEV)


def _run(shapes, Hq, Hkv, bs, window=0, sinks=None, seed=5):
    D = 128
    ctx = [c for _, c in shapes]
    ql = [a for a, _ in shapes]
    kc, vc, bt = _paged(ctx, Hkv, D, bs, seed)
    qs = [0]
    for a in ql[:-1]:
        qs.append(qs[-1] + a)
    q = torch.randn(sum(ql), (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    args = [torch.tensor(x, dtype=torch.int32, device=DEV) for x in (qs, ql, ctx)]
    return q, kc, vc, bt, args


@pytest.mark.parametrize("variant", ["1", "3", "7"])  # 1: builtin LDS-DMA, 3: asm LDS-DMA, 7: + pipelined halves
@pytest.mark.parametrize("Hq,Hkv", [(64, 8), (32, 8), (8, 8), (16, 8)])
@pytest.mark.parametrize("bs", [16, 64])
def test_prefill_v4_matches_reference(Hq, Hkv, bs, variant, monkeypatch):
    monkeypatch.setenv("LLMD_PREFILL_V4", "1")
    monkeypatch.setenv("LLMD_PREFILL_V4_VARIANT", variant)
    shapes = [(1, 1), (37, 37), (200, 200), (130, 1000), (64, 64), (513, 700)]
    q, kc, vc, bt, args = _run(shapes, Hq, Hkv, bs)
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 1 / math.sqrt(128))
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 1 / math.sqrt(128))
    _close(o, r)


def test_prefill_v4_window_sinks(monkeypatch):
    monkeypatch.setenv("LLMD_PREFILL_V4", "1")
    Hq, Hkv = 64, 8
    q, kc, vc, bt, args = _run([(300, 300), (77, 500)], Hq, Hkv, 64, seed=6)
    q = q[:, :Hq * 128].contiguous()
    sinks = torch.randn(Hq, device=DEV)
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 128 ** -0.5, 128, sinks)
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 128 ** -0.5, 128, sinks)
    _close(o, r)


@pytest.mark.parametrize("shapes", [[(5000, 5000)], [(2048, 8192), (3000, 5000)]])
def test_prefill_v4_long_vs_v2(shapes, monkeypatch):
    """Production shapes: v4 against v2 (itself checked against the chunked fp32 reference in
    tests/test_kernels_prod_shapes.py) - bf16-rounding close."""
    Hq, Hkv = 64, 8
    q, kc, vc, bt, args = _run(shapes, Hq, Hkv, 64, seed=3)
    scale = 1 / math.sqrt(128)
    monkeypatch.setenv("LLMD_PREFILL_V4", "0")
    o2 = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, scale)
    monkeypatch.setenv("LLMD_PREFILL_V4", "1")
    o4 = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, scale)
    assert torch.isfinite(o4.float()).all()
    _close(o4, o2, atol=2e-2, rtol=2e-2)
