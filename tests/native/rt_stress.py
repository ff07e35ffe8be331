"""Randomised stress / property driver for the native host runtime (_rt):
block manager (allocation, prefix caching, commit, free, remote allocation,
events, conservation invariant), precise KV-block index, approximate prefix
index, GBDT fit/predict/serialize, FS KV store.

Runs against any module object with the _rt API: the normal extension under
pytest (tests/test_rt_sanitize.py::test_stress_plain), and the ASan+UBSan
instrumented embedded build (tests/native/rt_sanitize_main.cpp) where every
out-of-bounds access / use-after-free / UB in the C++ aborts the run.
"""
import os
import random
import tempfile

import numpy as np


def stress_block_manager(rt, seed=0, iters=3000):
    rng = random.Random(seed)
    bs = 16
    bm = rt.BlockManager(64, bs, True, True)
    live = {}
    prompts = [np.array([rng.randrange(1, 50) for _ in range(rng.randrange(1, 200))], dtype=np.int32)
               for _ in range(20)]
    nid = 0
    for _ in range(iters):
        op = rng.random()
        if op < 0.35 and len(live) < 12:
            p = prompts[rng.randrange(len(prompts))]
            extra = rng.choice([0, 0, 7])
            hit = bm.lookup(p, extra)
            got = bm.acquire(nid, p, extra)
            assert got == hit and got % bs == 0 and got < max(1, len(p))
            live[nid] = [p, got, extra]
            nid += 1
        elif op < 0.65 and live:
            sid = rng.choice(list(live))
            p, done, _ = live[sid]
            step = rng.randrange(1, 64)
            tot = min(len(p) + 40, done + step)
            if bm.grow(sid, tot):
                toks = np.concatenate([p, np.arange(1, 41, dtype=np.int32)])[:tot]
                bm.commit(sid, toks, tot)
                live[sid][1] = tot
                assert bm.num_seq_blocks(sid) >= (tot + bs - 1) // bs
                tab = bm.block_table(sid)
                assert len(set(tab)) == len(tab) and all(0 <= b < 64 for b in tab)
        elif op < 0.85 and live:
            sid = rng.choice(list(live))
            bm.free(sid)
            del live[sid]
        elif op < 0.9:
            r = bm.allocate_remote(nid, rng.randrange(1, 300), 0)
            if r:
                live[nid] = [np.zeros(1, dtype=np.int32), len(r) * bs, 0]
            nid += 1
        elif op < 0.93:
            bm.take_events()
            bm.take_evicted()
        elif op < 0.94 and not live:
            bm.reset_prefix_cache()
        bm.check_invariants()
        assert 0.0 <= bm.usage() <= 1.0
    # all sequences' blocks are disjoint
    owned = [b for sid in live for b in bm.block_table(sid)]
    for sid in list(live):
        bm.free(sid)
    bm.check_invariants()
    assert bm.num_free() == 64
    return len(owned)


def stress_kv_index(rt, seed=1, iters=2000):
    rng = random.Random(seed)
    idx = rt.KVBlockIndex(5000, 4)
    pods = [f"10.0.0.{i}:8000" for i in range(6)]
    for _ in range(iters):
        keys = [rng.randrange(1, 400) for _ in range(rng.randrange(1, 30))]
        pod = rng.choice(pods)
        r = rng.random()
        if r < 0.5:
            idx.add(pod, keys, rng.choice(["gpu", "cpu"]))
        elif r < 0.7:
            idx.remove(pod, keys, "gpu")
        elif r < 0.75:
            idx.clear_pod(pod)
        elif r < 0.8:
            idx.add_speculative(pod, keys)
        else:
            s = idx.score(keys, pods)
            assert all(v >= 0 for v in dict(s).values()) if isinstance(s, dict) else True
    ap = rt.ApproxIndex(200)
    for i in range(iters):
        hs = [rng.randrange(1, 10**12) for _ in range(rng.randrange(1, 20))]
        srv = rng.choice(pods)
        ap.insert(srv, hs)
        ap.match(hs, pods)
        if i % 97 == 0:
            ap.remove_server(srv)
    rt.char_block_hashes("hello world " * 50, 16)
    return idx.size()


def stress_gbdt(rt, seed=2):
    rng = np.random.default_rng(seed)
    X = rng.random((400, 5))
    y = 3 * X[:, 0] + np.sin(6 * X[:, 1]) + 0.1 * rng.random(400)
    g = rt.GBDT(30, 4, 0.2, 5, 32, 0.0)
    g.fit(X, y)
    p = np.asarray(g.predict(X))
    assert p.shape == (400,) and np.abs(p - y).mean() < 0.5
    g2 = rt.GBDT()
    g2.deserialize(g.serialize())
    assert np.allclose(np.asarray(g2.predict(X)), p)
    return float(np.abs(p - y).mean())


def stress_fs_store(rt, seed=3):
    rng = np.random.default_rng(seed)
    with tempfile.TemporaryDirectory() as d:
        st = rt.FsStore(d, 4)
        blobs = {}
        for i in range(40):
            key = f"{int(rng.integers(1, 2**62)):016x}"
            data = rng.integers(0, 255, size=int(rng.integers(1, 5000)), dtype=np.uint8)
            st.write(key, data)
            blobs[key] = data
        st.flush()
        for k, v in blobs.items():
            assert st.exists(k)
            out = np.zeros_like(v)
            st.read(k, out)
            assert (out == v).all()
        for k in list(blobs)[:10]:
            st.remove(k)
            assert not st.exists(k)
    return len(blobs)


def stress_fs_overwrite(rt, seed=4, keys=3, rounds=300):
    """Zero-copy writes of the SAME names in quick succession (the offload tier
    re-storing a block): a ticket comes back exactly once, and once it is back
    the caller scribbles over its buffer (the host slot is reused) - that must
    never reach the file. The last write of each name wins."""
    import time

    rng = np.random.default_rng(seed)
    with tempfile.TemporaryDirectory() as d:
        st = rt.FsStore(d, 4)
        names = [f"{i:02x}{int(rng.integers(1, 2**40)):010x}" for i in range(keys)]
        bufs, live, last = {}, set(), {}
        for t in range(rounds):
            name = names[t % keys]
            b = np.full(4096 + 64 * (t % 7), t % 251, dtype=np.uint8)
            bufs[t] = b
            live.add(t)
            last[name] = b.copy()
            st.write_async(name, b.ctypes.data, b.nbytes, t)
            for done in st.poll_writes():
                assert done in live, done
                live.discard(done)
                bufs[done][:] = 255  # slot reused after the ticket came back
            if t % 37 == 0:
                time.sleep(0.001)
        st.flush()
        for done in st.poll_writes():
            assert done in live, done
            live.discard(done)
        assert not live, sorted(live)[:5]
        for name, want in last.items():
            out = np.zeros_like(want)
            assert st.read(name, out)
            assert (out == want).all(), name
    return rounds


def stress_epp_score(rt, seed=5, iters=3000):
    """EPP combine_pick: ragged-free random columns, every picker, n_pick past the candidate count."""
    rng = random.Random(seed)
    picks = 0
    for _ in range(iters):
        n = rng.randint(0, 40)
        cols = [[rng.uniform(-1, 2) for _ in range(n)] for _ in range(rng.randint(1, 6))]
        tot, idx = rt.combine_pick(cols, [rng.uniform(0, 3) for _ in cols], rng.randint(0, 3), rng.randint(0, 2),
                                   rng.getrandbits(64))
        assert len(tot) == n and len(set(idx)) == len(idx) and all(0 <= i < n for i in idx)
        picks += len(idx)
    try:
        rt.combine_pick([[1.0, 2.0], [1.0]], [1.0, 1.0], 1, 0, 1)
        raise AssertionError("ragged columns accepted")
    except ValueError:
        pass
    return picks


def run_all(rt):
    return {"bm": stress_block_manager(rt), "kv_index": stress_kv_index(rt), "gbdt_mae": stress_gbdt(rt),
            "fs": stress_fs_store(rt), "fs_overwrite": stress_fs_overwrite(rt), "epp_score": stress_epp_score(rt)}


if __name__ == "__main__":
    import importlib

    print(run_all(importlib.import_module(os.environ.get("RT_MODULE", "llmd_amd._rt"))))
