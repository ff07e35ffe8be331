"""Attention kernel numerics at the shapes the reference serves, against the
fp32 PyTorch reference (llmd_amd/ops/reference.py):

* ``--block-size 128`` (the AMD P/D recipe,
  /root/reference/guides/pd-disaggregation/modelserver/amd/vllm/base/patch-decode.yaml:16)
  next to 64;
* prefill at ISL 5000 and 8192 (BASELINE's P/D and prefix-cache configs), fresh
  and as a chunk over a cached prefix;
* decode up to 32k context (``--max-model-len 32000``) with batch 64-class
  mixes, through the split-K path and the device-side split size used by
  captured hipGraphs;
* fp8 (e4m3fn) KV with dequant scales at those shapes;
* MLA decode rows at 32k context.

The reference attention of a long prefill is evaluated in query chunks (same
causal result, bounded memory)."""
import math

import pytest
import torch

from llmd_amd import ops
from llmd_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
F8 = torch.float8_e4m3fn


def _close(a, b, atol=2e-2, rtol=2e-2):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=rtol)


def _paged(lens, Hkv, D, bs, fp8=False, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    nb_per = [(L + bs - 1) // bs for L in lens]
    total = sum(nb_per) + 3
    kv = torch.empty(total, 2, Hkv, bs, D, device=DEV, dtype=torch.bfloat16)
    kv.normal_(generator=torch.Generator(device=DEV).manual_seed(seed))
    if fp8:
        kv = (kv * 4).to(F8)  # use the e4m3 range; dequant scale 0.25 below
    kc, vc = kv[:, 0], kv[:, 1]
    perm = torch.randperm(total, generator=g)
    bt = torch.zeros(len(lens), max(nb_per) + 2, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nb_per):
        bt[i, :n] = perm[o:o + n].int()
        o += n
    return kc, vc, bt.to(DEV)


@pytest.mark.parametrize("bs", [64, 128])
@pytest.mark.parametrize("fp8", [False, True])
def test_decode_long_context(bs, fp8):
    Hq, Hkv, D = 64, 8, 128
    lens = [1, 127, 128, 129, 5000, 8192, 16385, 32000]
    kc, vc, bt = _paged(lens, Hkv, D, bs, fp8, seed=1)
    ks = vs = 0.25 if fp8 else 1.0
    B = len(lens)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    r = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, k_scale=ks, v_scale=vs)
    for split in [None, (1024, 32), (32000, 1)]:
        o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, split=split, max_ctx=max(lens),
                             k_scale=ks, v_scale=vs)
        _close(o, r)
    # captured-graph form: fixed grid of 64 splits, keys per split from the device
    o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, scale, split=(32768, 64), max_ctx=max(lens),
                         split_dev=torch.tensor([512], dtype=torch.int32, device=DEV), k_scale=ks, v_scale=vs)
    _close(o, r)


@pytest.mark.parametrize("bs", [64, 128])
def test_decode_batch_64_mixed(bs):
    """A decode batch of 64 at ~5k context (the P/D decode rank's step)."""
    Hq, Hkv, D = 64, 8, 128
    g = torch.Generator().manual_seed(5)
    lens = (4900 + torch.randint(0, 200, (64,), generator=g)).tolist()
    kc, vc, bt = _paged(lens, Hkv, D, bs, seed=2)
    q = torch.randn(64, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    r = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5)
    o = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5, max_ctx=max(lens))
    _close(o, r)


def _prefill_ref_chunked(q, kc, vc, bt, qs, ql, ctx, Hq, Hkv, D, scale, ks=1.0, vs=1.0, chunk=1024):
    out = torch.zeros(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    for i in range(len(ql)):
        first = ctx[i] - ql[i]
        for a in range(0, ql[i], chunk):
            b = min(ql[i], a + chunk)
            args = [torch.tensor([v], dtype=torch.int32, device=DEV) for v in (0, b - a, first + b)]
            out[qs[i] + a:qs[i] + b] = ref.paged_prefill(q[qs[i] + a:qs[i] + b], kc, vc, bt[i:i + 1], *args, Hq,
                                                         Hkv, D, scale, k_scale=ks, v_scale=vs)
    return out


@pytest.mark.parametrize("bs", [64, 128])
@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("shapes", [[(5000, 5000)], [(8192, 8192)], [(2048, 8192), (3000, 5000)]])
def test_prefill_long(bs, fp8, shapes):
    """Fresh ISL 5000 / 8192 prompts and chunks over cached prefixes (q_len, ctx)."""
    Hq, Hkv, D = 64, 8, 128
    ctx = [c for _, c in shapes]
    ql = [a for a, _ in shapes]
    kc, vc, bt = _paged(ctx, Hkv, D, bs, fp8, seed=3)
    ks = vs = 0.25 if fp8 else 1.0
    qs = [0]
    for a in ql[:-1]:
        qs.append(qs[-1] + a)
    q = torch.randn(sum(ql), (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    r = _prefill_ref_chunked(q, kc, vc, bt, qs, ql, ctx, Hq, Hkv, D, scale, ks, vs)
    args = [torch.tensor(x, dtype=torch.int32, device=DEV) for x in (qs, ql, ctx)]
    o = ops.paged_prefill(q, kc, vc, bt, *args, Hq, Hkv, D, scale, k_scale=ks, v_scale=vs)
    _close(o, r)


@pytest.mark.parametrize("fp8", [False, True])
def test_mla_decode_32k(fp8):
    """Absorbed MLA decode (DeepSeek: 128 heads, 512 latent + 64 rope) at 32k context."""
    H, bs = 128, 64
    lens = [1, 700, 8192, 32000]
    nb_per = [(L + bs - 1) // bs for L in lens]
    total = sum(nb_per) + 2
    cache = torch.randn(total, bs, 576, device=DEV, dtype=torch.bfloat16) * 0.5
    kv_scale = 1.0
    if fp8:
        cache = (cache * 4).to(F8)
        kv_scale = 0.25
    perm = torch.randperm(total)
    bt = torch.zeros(len(lens), max(nb_per) + 1, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nb_per):
        bt[i, :n] = perm[o:o + n].int()
        o += n
    bt = bt.to(DEV)
    q = torch.randn(len(lens), H * 576, device=DEV, dtype=torch.bfloat16)
    rows = torch.arange(len(lens), dtype=torch.int32, device=DEV)
    rl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    scale = 192 ** -0.5
    got = ops.mla_attention(q, cache, bt, rows, rl, H, scale, kv_scale=kv_scale)
    want = ref.mla_attention(q, cache, bt, rows, rl, H, scale, kv_scale)
    _close(got, want, atol=2e-2, rtol=3e-2)
