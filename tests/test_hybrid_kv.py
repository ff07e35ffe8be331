"""Hybrid KV-cache manager (engine/hybrid_kv.py; reference --no-disable-hybrid-
kv-cache-manager, guides/pd-disaggregation/modelserver/gpu/vllm/base/
patch-decode.yaml:19): sliding-window layers in their own small pool whose
out-of-window blocks are released every step.

* exact greedy tokens vs the same model with every layer on full-length KV
  (prompts far longer than the window, chunked prefill, decode past it);
* the windowed pool stays bounded by running sequences x window;
* prefix caching: a repeated prompt hits (its last window is still cached in
  the windowed pool) and gives the same tokens;
* capacity: at a fixed KV byte budget the full-attention pool holds ~L/L_full
  more tokens;
* the C++ block manager's window primitives (acquire_window / release_before,
  null block, conservation)."""
import numpy as np
import pytest

from llmd_amd import _rt_loader
from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams


def _engine(hybrid, **kw):
    opts = dict(device="cpu", block_size=16, num_gpu_blocks=96, max_num_batched_tokens=64, max_num_seqs=4,
                max_model_len=512, enforce_eager=True, hybrid_kv_cache_manager=hybrid, seed=5)
    opts.update(kw)
    return LLMEngine(EngineConfig.create("tiny-gpt-oss", **opts))


def _prompts():
    rng = np.random.default_rng(3)
    return [rng.integers(3, 500, size=n).tolist() for n in (150, 97, 40)]


def _run(eng, prompts, n=12):
    reqs = eng.generate(prompts, SamplingParams(max_tokens=n, temperature=0.0, ignore_eos=True))
    return [r.output_token_ids for r in reqs]


def test_hybrid_matches_full_kv_greedy():
    ref = _engine(False)
    assert not ref.runner.hybrid
    hyb = _engine(None)
    assert hyb.runner.hybrid and hyb.runner.kv_swa is not None
    assert hyb.runner.kv.shape[0] == 1 and hyb.runner.kv_swa.shape[0] == 1  # 1 full + 1 windowed layer
    assert _run(hyb, _prompts()) == _run(ref, _prompts())
    hyb.bm.check_invariants()


def test_windowed_pool_stays_bounded():
    eng = _engine(None)
    bm = eng.bm
    prompts = _prompts()
    for i, p in enumerate(prompts):
        eng.add_request(f"r{i}", p, SamplingParams(max_tokens=40, temperature=0.0, ignore_eos=True))
    peak = 0
    window_blocks = -(-16 // 16) + 2
    while eng.has_unfinished():
        eng.step()
        used = bm.swa.num_blocks - bm.swa.num_free()
        live = sum(len([b for b in bm.block_table_swa(r.seq_id) if b != 0]) for r in eng.sched.running)
        peak = max(peak, live)
        # a decoding sequence holds at most its window's blocks (+ the one being written)
        for r in eng.sched.running:
            if not r.is_prefill:
                assert len([b for b in bm.block_table_swa(r.seq_id) if b != 0]) <= window_blocks, r.seq_id
        assert used >= live
    # the full pool held every context token; the windowed pool only windows + chunks
    assert peak <= 4 * window_blocks + 64 // 16 + 4
    bm.check_invariants()


def test_hybrid_prefix_cache_hit():
    eng = _engine(None)
    p = _prompts()[0]
    a = _run(eng, [p])
    q0, h0 = eng.bm.prefix_stats()[1], eng.bm.prefix_stats()[0]
    b = _run(eng, [p])
    hits = eng.bm.prefix_stats()[0] - h0
    assert a == b
    assert hits >= 128  # most of the 150-token prompt came from the cache (both pools)
    ref = _run(_engine(False), [p])
    assert a == ref


def test_hybrid_capacity_at_fixed_budget():
    """At one KV byte budget the full-attention pool of a hybrid cache holds
    L / L_full as many tokens (2x for gpt-oss's alternating layers), minus the
    small windowed pool."""
    budget = 64 << 20
    plain = _engine(False, num_gpu_blocks=None, kv_cache_memory_bytes=budget)
    hyb = _engine(None, num_gpu_blocks=None, kv_cache_memory_bytes=budget, max_num_seqs=64,
                  max_num_batched_tokens=512)
    r = hyb.runner
    assert r.num_blocks * r.block_bytes() + r.num_swa_blocks * r.swa_block_bytes() <= budget + r.block_bytes()
    ratio = r.num_blocks / plain.runner.num_blocks
    assert 1.8 < ratio <= 2.0, ratio


def test_block_manager_window_primitives():
    rt = _rt_loader.rt()
    bm = rt.BlockManager(20, 4, True, False, 1)
    assert bm.num_blocks == 19 and bm.num_free() == 19
    t = np.arange(40, dtype=np.int32)
    assert bm.acquire_window(1, t, 0, 40, 6) == 0
    assert bm.grow(1, 40)
    bm.commit(1, t, 40)
    assert bm.release_before(1, 40 - 6 + 1) == 8       # blocks 0..7 end before key 35
    tab = bm.block_table(1)
    assert tab[:8] == [0] * 8 and 0 not in tab[8:]
    assert bm.release_before(1, 35) == 0                # idempotent
    bm.free(1)
    bm.check_invariants()
    assert bm.num_free() == 19
    # the last window of a 36-token prefix is still cached (LRU): hit with null entries before it
    assert bm.acquire_window(2, t, 0, 36, 6) == 36
    assert bm.block_table(2)[:7] == [0] * 7
    bm.check_invariants()
    with pytest.raises(RuntimeError):
        rt.BlockManager(8, 4, True, False, 0).release_before(1, 4)


@pytest.mark.gpu
def test_hybrid_gpu_graphs_match_full_kv():
    """On the GPU: the windowed layers read their own pool through the window-limited
    HIP decode / prefill kernels, eagerly and from captured decode hipGraphs
    (static windowed tables + slots), and produce the full-KV engine's tokens."""
    kw = dict(device="cuda", block_size=16, num_gpu_blocks=128, max_num_batched_tokens=128, max_num_seqs=8,
              max_model_len=1024, enforce_eager=False)
    ref = _engine(False, **kw)
    hyb = _engine(None, **kw)
    assert hyb.runner.hybrid and hyb.runner.graphs
    rng = np.random.default_rng(9)
    prompts = [rng.integers(3, 500, size=n).tolist() for n in (300, 129, 17, 64)]
    assert _run(hyb, prompts, n=40) == _run(ref, prompts, n=40)
    hyb.bm.check_invariants()


def _pd_engine(kt, **kw):
    return _engine(None, kv_transfer_config=kt, **kw)


@pytest.mark.parametrize("transport", ["tcp"])
@pytest.mark.parametrize("n_prompt", [150, 143])
def test_hybrid_pd_transfer_matches_aggregated(transport, n_prompt):
    """P/D between two hybrid caches (kvx moves the full pool's blocks and the
    windowed pool's last-window blocks): the decoder's tokens equal an aggregated
    full-KV engine's; the windowed table is null before the window on both sides;
    the prefiller frees both pools after the read. n_prompt 143 is the boundary
    case (n - window + 1) % bs == 0: the decoder's recomputed last prompt token
    attends key n - window, which lies in the block just below the one a query
    at position n would first need."""
    import time

    kt = {"kv_connector": "KvxConnector", "kv_role": "kv_both",
          "kv_connector_extra_config": {"transport": transport}}
    P, D = _pd_engine(kt), _pd_engine(kt)
    assert P.runner.hybrid and D.runner.hybrid
    ref = _engine(False)
    prompt = np.random.default_rng(11).integers(3, 500, size=n_prompt).tolist()

    def run(eng, rid, sp, ktp=None):
        r = eng.add_request(rid, prompt, sp, kv_transfer_params=ktp)
        for _ in range(20000):
            for o in eng.step():
                if o.request_id == rid and o.finished:
                    return r, o
            if eng.last_step_empty:
                time.sleep(0.001)
        raise AssertionError("request did not finish")

    _, op = run(P, "p", SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True), {"do_remote_decode": True})
    ktp = op.kv_transfer_params
    nb = -(-n_prompt // 16)
    assert len(ktp["remote_block_ids"]) == nb
    swa = ktp["remote_swa_block_ids"]
    lo = (n_prompt - 16) // 16  # window 16 in tiny-gpt-oss: the last window + the recomputed token's key
    assert swa[:lo] == [0] * lo and 0 not in swa[lo:]
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    rd, od = run(D, "d", sp, ktp)
    want = ref.generate([prompt], sp)[0].output_token_ids
    assert rd.output_token_ids == want
    for _ in range(300):
        P.step()
        if P.bm.num_free() == P.bm.num_blocks and P.bm.swa.num_free() == P.bm.swa.num_blocks:
            break
    assert P.bm.num_free() == P.bm.num_blocks and P.bm.swa.num_free() == P.bm.swa.num_blocks
    P.bm.check_invariants()
    D.bm.check_invariants()


@pytest.mark.parametrize("tier", ["cpu", "fs"])
def test_hybrid_tiered_offload_reload(tier, tmp_path):
    """Tiered offload of a hybrid cache: both pools store write-through (host slots
    split by block bytes, FS keys of the windowed pool suffixed), a reload after the
    GPU prefix cache is dropped brings back the full pool's prefix and the windowed
    pool's last window, and the tokens equal a full-KV engine's."""
    kw = {"cpu_bytes_to_use": 64 << 20}
    if tier == "fs":
        kw["fs_root"] = str(tmp_path / "kv")
    prompt = np.random.default_rng(21).integers(3, 500, size=150).tolist()
    sp = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True)
    want = _engine(False).generate([prompt], sp)[0].output_token_ids
    eng = _engine(None, kv_offload_config=kw)
    assert eng.runner.hybrid
    assert eng.generate([prompt], sp)[0].output_token_ids == want
    off = eng.offload
    off.full.poll()
    off.swa.poll()
    assert off.full.stats["offloaded"] >= 150 // 16 and off.swa.stats["offloaded"] >= 150 // 16
    if tier == "fs":
        off.full.fs.flush()
        off.swa.fs.flush()
        eng = _engine(None, kv_offload_config=kw)  # fresh engine: empty GPU + host tiers
        off = eng.offload
    else:
        eng.reset_prefix_cache()
    assert eng.generate([prompt], sp)[0].output_token_ids == want
    key = "loaded_cpu" if tier == "cpu" else "loaded_fs"
    assert off.full.stats[key] >= 150 // 16 - 1
    assert 1 <= off.swa.stats[key] <= 3  # only the last window of the windowed pool
    eng.bm.check_invariants()


def test_hybrid_grow_is_all_or_nothing_when_windowed_pool_exhausted():
    """A windowed pool smaller than the full one runs out first: grow fails
    without keeping the full pool's new blocks, can_allocate sees the windowed
    pool, and freeing a sequence makes the grow succeed."""
    from llmd_amd.engine.hybrid_kv import HybridBlockManager

    rt = _rt_loader.rt()
    bm = HybridBlockManager(rt, num_full_blocks=64, num_swa_blocks=6, block_size=16, window=16,
                            prefix_caching=False, emit_events=False)
    toks = np.arange(3, 200, dtype=np.int32)
    assert bm.acquire(1, toks, 0) == 0 and bm.acquire(2, toks, 0) == 0
    assert bm.grow(1, 64)                      # 4 blocks in each pool (swa: 5 usable after the null)
    free_full, free_swa = bm.full.num_free(), bm.swa.num_free()
    assert free_swa == 1
    assert not bm.can_allocate(2)              # the full pool could, the windowed pool cannot
    assert not bm.grow(2, 32)                  # needs 2 windowed blocks, 1 free
    assert bm.full.num_free() == free_full and bm.swa.num_free() == free_swa
    assert bm.full.num_seq_blocks(2) == 0
    bm.after_compute(1, 64)                    # window 16: blocks below (64-16+1)//16 = 3 go back
    assert bm.swa.num_free() == 4
    assert bm.grow(2, 32) and bm.full.num_seq_blocks(2) == 2 and bm.swa.num_seq_blocks(2) == 2
    bm.free(1)
    bm.free(2)
    bm.check_invariants()
