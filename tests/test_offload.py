"""Tiered KV offload: host-DRAM write-through + reload, and
the filesystem tier surviving an engine restart. CPU engine, exact-token
equality against a run without offload."""
import numpy as np

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
