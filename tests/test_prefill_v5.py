"""Prefill attention v5 (csrc/ops/attn_prefill5.hip: v2's tiles with the QK product of tile t+1
and the softmax of tile t software-pipelined inside a wave, K / V in separate LDS rings) against
the fp32 reference - fresh prompts, chunks over cached prefixes (partial last tiles), GQA groups
of 4 and 8, blocks of 64 and 128 keys, sinks - and against v2 at the production ISL 5000 /
8192 shapes. Shapes v5 does not cover (window, D 64, blocks of 16, GQA 1 / 2) fall back to v2."""
import math

import pytest
import torch

from llmd_amd import ops
from llmd_amd.ops import reference as ref

from test_prefill_v4 import _close, _run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Hq,Hkv", [(64, 8), (32, 8), (32, 4)])
@pytest.mark.parametrize("bs", [64, 128])
def test_prefill_v5_matches_reference(Hq, Hkv, bs, monkeypatch):
    monkeypatch.setenv("LLMD_PREFILL_V5", "1")
    shapes = [(1, 1), (37, 37), (200, 200), (130, 1000), (64, 64), (513, 700), (65, 129)]
    q, kc, vc, bt, args = _run(shapes, Hq, Hkv, bs)
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 1 / math.sqrt(128))
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 1 / math.sqrt(128))
    _close(o, r)


def test_prefill_v5_sinks_and_fallbacks(monkeypatch):
    monkeypatch.setenv("LLMD_PREFILL_V5", "1")
    Hq, Hkv = 64, 8
    q, kc, vc, bt, args = _run([(300, 300), (77, 500)], Hq, Hkv, 64, seed=6)
    q = q[:, :Hq * 128].contiguous()
    sinks = torch.randn(Hq, device="cuda")
    for window in (0, 128):  # 128: sliding window -> v2
        r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 128 ** -0.5, window, sinks)
        o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 128 ** -0.5, window, sinks)
        _close(o, r)
    q, kc, vc, bt, args = _run([(100, 300)], 16, 8, 16, seed=7)  # GQA 2, blocks of 16 -> v2
    _close(ops.paged_prefill(q, kc, vc, bt, *args, 16, 8, 128, 128 ** -0.5),
           ref.paged_prefill(q, kc, vc, bt, *args, 16, 8, 128, 128 ** -0.5))


@pytest.mark.parametrize("shapes", [[(5000, 5000)], [(2048, 8192), (3000, 5000)]])
def test_prefill_v5_long_vs_v2(shapes, monkeypatch):
    Hq, Hkv = 64, 8
    q, kc, vc, bt, args = _run(shapes, Hq, Hkv, 64, seed=3)
    scale = 1 / math.sqrt(128)
    monkeypatch.setenv("LLMD_PREFILL_V5", "0")
    o2 = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, scale)
    monkeypatch.setenv("LLMD_PREFILL_V5", "1")
    o5 = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, scale)
    assert torch.isfinite(o5.float()).all()
    _close(o5, o2, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("variant", ["53", "181", "309", "437"])
@pytest.mark.parametrize("Hq,Hkv,bs", [(64, 8, 64), (32, 8, 16), (8, 8, 64)])
def test_prefill_v2_variants_match_reference(variant, Hq, Hkv, bs, monkeypatch):
    """v2 schedule variants (LLMD_PREFILL_V2_VARIANT): 53 = round-6 default; + 128: Q pre-scaled and
    the S^T accumulators started at -m (no per-score v_fma); + 256: row sums as P . ones MFMAs."""
    monkeypatch.setenv("LLMD_PREFILL_V5", "0")
    monkeypatch.setenv("LLMD_PREFILL_V2_VARIANT", variant)
    shapes = [(1, 1), (37, 37), (200, 200), (130, 1000), (64, 64), (513, 700), (65, 129)]
    q, kc, vc, bt, args = _run(shapes, Hq, Hkv, bs)
    r = ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 1 / math.sqrt(128))
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, 128, 1 / math.sqrt(128))
    _close(o, r)
    sinks = torch.randn(Hq, device="cuda")
    q2 = q[:, :Hq * 128].contiguous()
    for window in (0, 128):
        _close(ops.paged_prefill(q2, kc, vc, bt, *args, Hq, Hkv, 128, 128 ** -0.5, window, sinks),
               ref.paged_prefill(q2, kc, vc, bt, *args, Hq, Hkv, 128, 128 ** -0.5, window, sinks))


@pytest.mark.parametrize("variant", ["5", "53", "181", "437"])
@pytest.mark.parametrize("window", [0, 128])
def test_prefill_v2_variants_d64_match_reference(variant, window, monkeypatch):
    """The gpt-oss attention shape (64 / 8 heads, D 64, sliding window 128 on half the layers,
    sinks) under each v2 variant instantiated for D = 64."""
    monkeypatch.setenv("LLMD_PREFILL_V2_VARIANT", variant)
    torch.manual_seed(11)
    Hq, Hkv, D, bs = 64, 8, 64, 64
    shapes = [(1, 1), (37, 37), (200, 200), (130, 1000), (513, 700), (65, 129)]
    ctx = [c for _, c in shapes]
    ql = [a for a, _ in shapes]
    nb = [(c + bs - 1) // bs for c in ctx]
    total = sum(nb) + 3
    kc = torch.randn(total, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(total, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    perm = torch.randperm(total)
    bt = torch.zeros(len(ctx), max(nb) + 1, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nb):
        bt[i, :n] = perm[o:o + n].int()
        o += n
    bt = bt.cuda()
    qs = [0]
    for a in ql[:-1]:
        qs.append(qs[-1] + a)
    q = torch.randn(sum(ql), Hq * D, device="cuda", dtype=torch.bfloat16)
    args = [torch.tensor(x, dtype=torch.int32, device="cuda") for x in (qs, ql, ctx)]
    sinks = torch.randn(Hq, device="cuda")
    _close(ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, D ** -0.5, window, sinks),
           ref.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, D ** -0.5, window, sinks))
