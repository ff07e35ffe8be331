"""Tiered KV offload: host-DRAM write-through + reload, and
the filesystem tier surviving an engine restart. CPU engine, exact-token
equality against a run without offload."""
import numpy as np
import pytest

from llmd_amd.engine.request import SamplingParams
from tests.test_engine import make_engine


def _gen(eng, prompt, n=8):
    outs = eng.generate([prompt], SamplingParams(max_tokens=n, temperature=0.0, ignore_eos=True))
    return list(outs[0].output_token_ids)


def _prompt(seed=7, n=150):
    return np.random.default_rng(seed).integers(3, 500, size=n).tolist()


def test_host_offload_reload_exact():
    base = _gen(make_engine(), _prompt())
    eng = make_engine(kv_offload_config={"cpu_bytes_to_use": 64 << 20})
    assert _gen(eng, _prompt()) == base
    off = eng.offload
    assert off.stats["offloaded"] >= 150 // 16
    eng.reset_prefix_cache()  # drop the GPU-tier prefix cache
    out = _gen(eng, _prompt())
    assert out == base
    assert off.stats["loaded_cpu"] >= 150 // 16 - 1
    evs = off.take_events()
    assert all(e[5] == "cpu" for e in evs)


def test_host_lru_eviction_events():
    eng = make_engine(kv_offload_config={"cpu_bytes_to_use": 1})  # one host slot
    _gen(eng, _prompt(n=80))
    eng.offload.poll()
    assert eng.offload.stats["evicted_cpu"] > 0
    assert len(eng.offload.slot_of) == 1


def test_fs_tier_survives_restart(tmp_path):
    base = _gen(make_engine(), _prompt(3))
    cfg = {"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}
    eng = make_engine(kv_offload_config=cfg)
    assert _gen(eng, _prompt(3)) == base
    eng.offload.fs.flush()
    assert eng.offload.fs.written >= 150 // 16
    eng2 = make_engine(kv_offload_config=cfg)  # fresh engine, empty GPU + host tiers
    assert _gen(eng2, _prompt(3)) == base
    assert eng2.offload.stats["loaded_fs"] >= 150 // 16 - 1


def test_host_reload_retried_when_pool_was_full():
    """A request whose prefix is in the host tier but arrives while the GPU
    pool is full gets its reload when it is admitted later (not a from-scratch
    prefill), and generates the same tokens."""
    p, blocker = _prompt(11, 96), _prompt(12, 150)
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    base = _gen(make_engine(num_gpu_blocks=16), p)
    eng = make_engine(num_gpu_blocks=16, kv_offload_config={"cpu_bytes_to_use": 64 << 20})
    assert _gen(eng, p) == base                  # p's blocks are written through to the host tier
    eng.reset_prefix_cache()
    eng.add_request("blocker", blocker, SamplingParams(max_tokens=40, temperature=0.0, ignore_eos=True))
    eng.step()                                   # blocker takes 10+ of the 16 blocks
    eng.add_request("again", p, sp)
    outs = {"again": [], "blocker": []}
    for _ in range(500):
        if not eng.has_unfinished():
            break
        for o in eng.step():
            outs[o.request_id] += o.new_token_ids
    assert not eng.has_unfinished()  # a waiting request holding blocks used to deadlock here
    assert outs["again"] == base
    assert eng.offload.stats["loaded_cpu"] >= 96 // 16 - 1
    # while the pool cannot hold it, the waiting request does not reload (and give back)
    # its host prefix every step: one reload, not one per blocked step
    assert eng.offload.stats["loaded_cpu"] <= 2 * (96 // 16)


def test_offload_metrics_use_vllm_names(tmp_path):
    """Transfer metrics follow vLLM's offloading contract (vllm:kv_offload_*: bytes,
    time and size distribution per transfer type; kv-offloader.md:211)."""
    cfg = {"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}
    eng = make_engine(kv_offload_config=cfg)
    _gen(eng, _prompt(5))
    eng.offload.fs.flush()
    eng.reset_prefix_cache()
    _gen(eng, _prompt(5))
    text = eng.offload.render_metrics("m").decode()
    assert "llmd:kv_offload" not in text
    for t in ("GPU_to_CPU", "CPU_to_GPU", "CPU_to_FS"):
        line = next(l for l in text.splitlines()
                    if l.startswith("vllm:kv_offload_total_bytes") and f'transfer_type="{t}"' in l)
        assert float(line.split()[-1]) > 0, line
    assert 'vllm:kv_offload_size_bucket{model_name="m",transfer_type="GPU_to_CPU",le="+Inf"}' in text
    assert 'vllm:kv_offload_total_time{model_name="m",transfer_type="CPU_to_GPU"}' in text


def test_fs_reload_is_asynchronous(tmp_path):
    """An FS-tier reload does not read the disk on the engine thread: the request
    waits in offload_wait while the native read pool fills pinned buffers, and
    other requests keep being scheduled meanwhile."""
    cfg = {"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}
    base = _gen(make_engine(), _prompt(9))
    eng = make_engine(kv_offload_config=cfg)
    _gen(eng, _prompt(9))
    eng.offload.fs.flush()
    eng2 = make_engine(kv_offload_config=cfg)
    fs = eng2.offload.fs
    reads = []
    orig = fs.read
    fs_read_sync = []

    class Spy:  # the synchronous read must never be used by the engine
        def __getattr__(self, k):
            if k == "read":
                fs_read_sync.append(1)
            return getattr(fs, k)
    eng2.offload.fs = Spy()
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    eng2.add_request("fs", _prompt(9), sp)
    eng2.add_request("other", _prompt(10, 40), SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    outs = {"fs": [], "other": []}
    for o in eng2.step():
        outs[o.request_id] += o.new_token_ids
    assert "fs" in eng2.sched.offload_wait or eng2.offload.stats["loaded_fs"] > 0
    for _ in range(200):
        if not eng2.has_unfinished():
            break
        for o in eng2.step():
            outs[o.request_id] += o.new_token_ids
    assert outs["fs"] == base and len(outs["other"]) == 4
    assert eng2.offload.stats["loaded_fs"] >= 150 // 16 - 1
    assert not fs_read_sync and not reads and orig


def test_fs_reload_joins_host_tier(tmp_path):
    """An FS reload reads into host-tier slots (no per-block pinned buffers) and
    those blocks stay in the host tier: the next reload of the same prefix is
    served from host memory, not from disk."""
    cfg = {"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}
    base = _gen(make_engine(), _prompt(14))
    eng = make_engine(kv_offload_config=cfg)
    _gen(eng, _prompt(14))
    eng.offload.fs.flush()
    eng2 = make_engine(kv_offload_config=cfg)
    assert _gen(eng2, _prompt(14)) == base
    off = eng2.offload
    n_fs = off.stats["loaded_fs"]
    assert n_fs >= 150 // 16 - 1
    assert len(off.slot_of) >= n_fs and not any(off.slot_busy.values())
    eng2.reset_prefix_cache()
    assert _gen(eng2, _prompt(14)) == base
    assert off.stats["loaded_fs"] == n_fs and off.stats["loaded_cpu"] >= n_fs


def test_invalidate_cancels_inflight_reload(tmp_path):
    """A weight update while an FS reload is in flight: the reload
    reports 0 tokens (the request recomputes its prefix), its host-slot
    references are released exactly once (no negative busy counts, every slot
    can be recycled), and the request still completes with the right tokens."""
    cfg = {"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}
    base = _gen(make_engine(), _prompt(15))
    eng = make_engine(kv_offload_config=cfg)
    _gen(eng, _prompt(15))
    eng.offload.fs.flush()
    eng2 = make_engine(kv_offload_config=cfg)
    off = eng2.offload
    eng2.add_request("x", _prompt(15), SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
    eng2.sched.schedule()
    assert "x" in eng2.sched.offload_wait and off.loads
    off.invalidate("new-weights")
    assert all(v == 0 for v in off.slot_busy.values())
    out = []
    for _ in range(300):
        if not eng2.has_unfinished():
            break
        for o in eng2.step():
            out += o.new_token_ids
    assert out == base
    assert off.stats["loaded_fs"] == 0
    assert all(v >= 0 for v in off.slot_busy.values())
    assert len(off.free_slots) + len(off.slot_of) == off.n_slots


def test_abort_while_loading_frees_blocks():
    eng = make_engine(kv_offload_config={"cpu_bytes_to_use": 64 << 20})
    _gen(eng, _prompt(13))
    eng.reset_prefix_cache()
    free0 = eng.bm.num_free()
    eng.add_request("x", _prompt(13), SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    eng.sched.schedule()  # admission starts the reload (CPU engine: it completes at once)
    if "x" in eng.sched.offload_wait:
        eng.abort("x")
        eng.sched.schedule()
        assert "x" not in eng.sched.offload_wait
        assert eng.bm.num_free() == free0


@pytest.mark.gpu
def test_gpu_offload_pack_unpack_roundtrip(tmp_path):
    """GPU pool: write-through packs blocks with the LDS-staged copy kernel on the
    side stream, D2H into pinned slots, and the asynchronous reload (H2D + unpack
    kernel) restores the exact KV: same greedy tokens, and the reloaded blocks
    are bit-identical to the ones computed by prefill."""
    import torch

    cfg = {"cpu_bytes_to_use": 256 << 20, "fs_root": str(tmp_path / "kv")}
    eng = make_engine(device="cuda", kv_offload_config=cfg, num_gpu_blocks=128)
    p = _prompt(21, 300)
    base = _gen(eng, p)
    eng.offload._drain()
    keys = list(eng.offload.slot_of)
    assert len(keys) >= 300 // 16 - 1
    before = eng.offload.host[[eng.offload.slot_of[k] for k in keys]].clone()
    eng.reset_prefix_cache()
    assert _gen(eng, p) == base
    assert eng.offload.stats["loaded_cpu"] >= 300 // 16 - 1
    eng.offload.fs.flush()
    eng2 = make_engine(device="cuda", kv_offload_config=cfg, num_gpu_blocks=128)  # FS tier only
    assert _gen(eng2, p) == base
    assert eng2.offload.stats["loaded_fs"] >= 300 // 16 - 1
    # the reloaded blocks are written through again: disk -> H2D -> unpack -> pack -> D2H
    # must give back the original bytes
    eng2.offload._drain()
    common = [k for k in keys if k in eng2.offload.slot_of]
    assert len(common) >= 300 // 16 - 1
    a = torch.stack([before[keys.index(k)] for k in common])
    b = eng2.offload.host[[eng2.offload.slot_of[k] for k in common]]
    assert torch.equal(a, b)
