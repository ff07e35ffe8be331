"""Property-based tests (hypothesis): block-hash chain and
approximate char-block hashes are prefix-stable, and the native block
allocator conserves blocks (free + referenced == total) under arbitrary
acquire / grow / commit / free interleavings; the precise index's scores are
monotone in the matched prefix."""
import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from llmd_amd import _rt_loader

rt = _rt_loader.rt()
toks = st.lists(st.integers(1, 1000), min_size=0, max_size=300)


@given(toks, toks, st.sampled_from([16, 64]), st.integers(0, 3))
@settings(max_examples=60, deadline=None)
def test_hash_chain_prefix_stable(a, b, bs, extra):
    ha = list(rt.hash_blocks(a, bs, extra))
    hab = list(rt.hash_blocks(a + b, bs, extra))
    assert len(ha) == len(a) // bs
    assert hab[:len(ha)] == ha                     # a prefix's keys never change
    if ha and extra != 1:
        assert list(rt.hash_blocks(a, bs, 1))[0] != ha[0]   # extra keys (LoRA/mm) separate namespaces


@given(st.text(min_size=0, max_size=400), st.text(max_size=200), st.sampled_from([8, 64]))
@settings(max_examples=60, deadline=None)
def test_char_block_hashes_prefix_stable(a, b, bc):
    ha = list(rt.char_block_hashes(a, bc))
    hab = list(rt.char_block_hashes(a + b, bc))
    assert hab[:len(ha)] == ha


ops = st.lists(st.tuples(st.sampled_from(["acq", "grow", "commit", "free"]), st.integers(0, 7),
                         st.integers(1, 120)), min_size=1, max_size=80)


@given(ops, st.booleans())
@settings(max_examples=80, deadline=None)
def test_allocator_conservation(seq, caching):
    bs, nb = 16, 24
    bm = rt.BlockManager(nb, bs, caching, False)
    live = {}
    base = np.arange(1, 400, dtype=np.int32) % 37
    for op, sid, n in seq:
        if op == "acq" and sid not in live:
            p = base[:n].copy()
            hit = bm.acquire(sid, p, 0)
            assert hit % bs == 0 and hit <= max(0, n - 1)
            live[sid] = [p, hit]
        elif op == "grow" and sid in live:
            tot = live[sid][1] + n
            if bm.grow(sid, tot):
                live[sid][1] = tot
        elif op == "commit" and sid in live:
            p, done = live[sid]
            bm.commit(sid, np.resize(p, max(done, 1)).astype(np.int32), done)
        elif op == "free" and sid in live:
            bm.free(sid)
            del live[sid]
        bm.check_invariants()
        owned = [b for s in live for b in bm.block_table(s)]
        # distinct referenced blocks + free (incl. cached-evictable) never exceed the pool
        assert len(set(owned)) + bm.num_free() <= nb
    for s in list(live):
        bm.free(s)
    bm.check_invariants()
    assert bm.num_free() == nb


@given(st.integers(1, 30), st.integers(0, 30))
@settings(max_examples=40, deadline=None)
def test_index_score_monotone_in_prefix(n, m):
    idx = rt.KVBlockIndex(10000, 4)
    keys = list(range(100, 100 + max(n, m)))
    idx.add("a:1", keys[:n])
    idx.add("b:1", keys[:m])
    s = dict(idx.score(keys, ["a:1", "b:1"]))
    if n > m:
        assert s.get("a:1", 0) >= s.get("b:1", 0)
    elif m > n:
        assert s.get("b:1", 0) >= s.get("a:1", 0)
