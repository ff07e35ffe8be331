"""Shared-prefix (cascade) decode plan: grouping by shared physical blocks,
work-unit coverage, and the decomposition math (prefix partial from the
item's first member's blocks + own suffix, merged by log-sum-exp) against the
plain fp32 decode reference (CPU)."""
import numpy as np
import pytest
import torch

from llmd_amd import ops
from llmd_amd.ops import reference as ref
from shared_prefix_util import shared_tables


def _lse_merge(parts):
    m = torch.stack([p[1] for p in parts]).amax(0)
    num = sum(p[0] * torch.exp(p[1] - m)[..., None] for p in parts)
    den = sum(p[2] * torch.exp(p[1] - m) for p in parts)
    return num / den[..., None]


def _partial(q, k, v, scale):
    """q [H, D], k/v [n, Hkv, D] (GQA) -> (unnormalised O [H, D], max [H], sum [H])."""
    H, Hkv = q.shape[0], k.shape[1]
    kk = k.repeat_interleave(H // Hkv, 1).permute(1, 0, 2)
    vv = v.repeat_interleave(H // Hkv, 1).permute(1, 0, 2)
    s = torch.einsum("hd,hnd->hn", q, kk) * scale
    m = s.amax(-1)
    p = torch.exp(s - m[:, None])
    return torch.einsum("hn,hnd->hd", p, vv), m, p.sum(-1)


def _gather(cache, row, lo, hi, bs):
    idx = torch.arange(lo, hi)
    blocks = torch.as_tensor(row)[idx // bs].long()
    return cache[blocks, :, idx % bs]  # [n, Hkv, D]


def test_plan_groups_and_covers():
    bs = 16
    bt, lens, _ = shared_tables([(640, 3), (320, 5), (1024, 1), (48, 2)], [1, 17, 200, 33], bs)
    plan = ops.shared_prefix_plan(bt, lens, bs, G=8, Hkv=8, variant=2, min_prefix=256, min_chunk=128)
    assert plan is not None
    cap = 32 // 8  # variant 2: two 16-column passes of 2 members at G = 8
    for b in range(len(lens)):
        P = int(plan.sstart[b])
        assert P % bs == 0 and P <= lens[b] - 1
    # the 1024-token singleton and the 48-token pair (below min_prefix) are not shared
    assert plan.sstart[8] == 0 and plan.sstart[9] == 0 and plan.sstart[10] == 0
    assert (plan.sstart[:8] > 0).all()
    seen = {}
    for m0, nm, lo, hi, slot in plan.work.tolist():
        if nm == 0:
            continue
        assert 2 <= nm <= cap
        mem = plan.members[m0:m0 + nm].tolist()
        first = bt[mem[0]]
        P = int(plan.sstart[mem[0]])
        for b in mem:
            assert plan.sstart[b] == P
            assert (bt[b, :P // bs] == first[:P // bs]).all()  # really the same physical blocks
        seen.setdefault(tuple(mem), []).append((lo, hi, slot))
    for mem, ranges in seen.items():
        ranges.sort()
        P = int(plan.sstart[mem[0]])
        assert ranges[0][0] == 0 and ranges[-1][1] == P
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
        assert [r[2] for r in ranges] == list(range(len(ranges)))
        assert all(plan.pcount[b] == len(ranges) for b in mem)


def test_cascade_variant():
    assert ops.cascade_variant(8, 128, 64, False) == 3
    assert ops.cascade_variant(4, 64, 128, False) == 3
    assert ops.cascade_variant(8, 128, 16, False) == 3  # 64-key tiles over four blocks
    assert ops.cascade_variant(8, 64, 4, False) == 1    # a DMA instruction's rows span blocks
    assert ops.cascade_variant(8, 128, 64, True) == 1   # fp8 cache: register kernel
    assert ops.cascade_variant(2, 64, 64, False) == 1
    assert ops.cascade_variant(16, 128, 64, False) == 2
    assert ops.cascade_variant(5, 128, 64, False) is None


def test_plan_none_without_sharing():
    bt, lens, _ = shared_tables([(0, 1)] * 6, [700], 16)
    assert ops.shared_prefix_plan(bt, lens, 16, G=8) is None
    assert ops.shared_prefix_plan(bt[:1], lens[:1], 16, G=8) is None
    bt, lens, _ = shared_tables([(640, 3)], [5], 16)
    assert ops.shared_prefix_plan(bt, lens, 16, G=5) is None  # 16 % G != 0: plain path


def test_plan_respects_work_capacity():
    bt, lens, _ = shared_tables([(2048, 2)] * 6, [40], 64)
    plan = ops.shared_prefix_plan(bt, lens, 64, G=8, Hkv=8, max_work=5, min_chunk=512)
    assert plan.work.shape == (5, 5)
    used = plan.work[plan.work[:, 1] > 0]
    assert len(used) <= 5
    shared = {int(b) for m0, nm, *_ in used.tolist() for b in plan.members[m0:m0 + nm]}
    assert all((plan.sstart[b] > 0) == (b in shared) for b in range(len(lens)))


@pytest.mark.parametrize("variant", [1, 2, 3])
@pytest.mark.parametrize("G,groups", [(8, [(512, 2), (256, 4), (768, 3), (512, 17)]), (4, [(384, 7), (512, 2)]),
                                      (16, [(640, 2)])])
def test_cascade_decomposition_matches_decode(G, groups, variant):
    if ops.CASCADE_MEMBERS[variant](G) < 2:
        pytest.skip("one member per item: nothing to share")
    torch.manual_seed(0)
    bs, Hkv, D = 16, 2, 32
    Hq = Hkv * G
    bt, lens, nb = shared_tables(groups, [1, 9, 31, 100], bs, seed=1)
    kc = torch.randn(nb, Hkv, bs, D)
    vc = torch.randn(nb, Hkv, bs, D)
    B = len(lens)
    q = torch.randn(B, Hq * D)
    scale = D ** -0.5
    plan = ops.shared_prefix_plan(bt, lens, bs, G=G, Hkv=Hkv, variant=variant, min_prefix=128, min_chunk=64)
    assert plan is not None and plan.items >= 1
    cap = ops.CASCADE_MEMBERS[variant](G)
    assert all(nm <= cap for nm in plan.work[:, 1])
    want = ref.paged_decode(q, kc, vc, torch.from_numpy(bt), torch.from_numpy(lens), Hq, Hkv, D, scale)
    parts = {b: [] for b in range(B)}
    for m0, nm, lo, hi, slot in plan.work.tolist():
        if nm == 0:
            continue
        mem = plan.members[m0:m0 + nm].tolist()
        k = _gather(kc, bt[mem[0]], lo, hi, bs)  # the prefix is read through the first member's table
        v = _gather(vc, bt[mem[0]], lo, hi, bs)
        for b in mem:
            parts[b].append(_partial(q[b].view(Hq, D), k, v, scale))
    for b in range(B):
        s0 = int(plan.sstart[b])
        k = _gather(kc, bt[b], s0, int(lens[b]), bs)
        v = _gather(vc, bt[b], s0, int(lens[b]), bs)
        parts[b].append(_partial(q[b].view(Hq, D), k, v, scale))
        assert len(parts[b]) == 1 + int(plan.pcount[b])
        got = _lse_merge(parts[b]).reshape(-1)
        torch.testing.assert_close(got, want[b].float(), atol=1e-4, rtol=1e-4)


def test_cascade_tensor_layout():
    bt, lens, _ = shared_tables([(640, 3)], [5, 70], 16)
    plan = ops.shared_prefix_plan(bt, lens, 16, G=8, min_prefix=256, min_chunk=128)
    t, np_, slots = ops.cascade_tensors(plan, "cpu")
    B = len(lens)
    assert t.dtype == torch.int32 and t.numel() == 3 * B + plan.work.size
    assert np.array_equal(t[:B].numpy(), plan.sstart) and np_ == plan.np and slots == plan.max_slots
    assert np.array_equal(t[3 * B:].view(-1, 5).numpy(), plan.work)


def _shared_prefix_run(device, monkeypatch, model="tiny-llama", **kw):
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    calls = []
    real = ops.shared_prefix_plan

    def counting(*a, **k):
        p = real(*a, **k)
        calls.append(p is not None and p.items > 0)
        return p

    monkeypatch.setattr(ops, "shared_prefix_plan", counting)
    cfg = EngineConfig.create(model, device=device, block_size=16, num_gpu_blocks=256,
                              max_num_batched_tokens=1024, max_num_seqs=8, max_model_len=2048,
                              cuda_graph_max_bs=8, **kw)
    eng = LLMEngine(cfg)
    prefix = [(7 * i) % 500 + 3 for i in range(700)]
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    eng.generate([prefix + [9]], SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))  # cache it
    prompts = [prefix + [20 + i] * (1 + 5 * i) for i in range(6)] + [[5 + i for i in range(300)]]
    outs = [r.output_token_ids for r in eng.generate(prompts, sp)]
    return eng, prompts, outs, any(calls)


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-gpt-oss"])
def test_engine_shared_prefix_decode_cpu(monkeypatch, model):
    """The engine groups the decode rows that share the cached prefix (CPU:
    the reference attention ignores the plan, so outputs are unchanged)."""
    _, _, a, used = _shared_prefix_run("cpu", monkeypatch, model)
    assert used
    _, _, b, used_off = _shared_prefix_run("cpu", monkeypatch, model, shared_prefix_decode=False)
    assert not used_off and a == b
