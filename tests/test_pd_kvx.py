"""P/D disaggregation through kvx on CPU (TCP transport) and failure policies."""
import os

import numpy as np
import pytest

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams


def make(kt=None, **kw):
    cfg = EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=128,
                              max_num_batched_tokens=128, max_num_seqs=8, max_model_len=512,
                              enforce_eager=True, kv_transfer_config=kt, seed=0, **kw)
    return LLMEngine(cfg)


def run(eng, rid, prompt, sp, ktp=None):
    r = eng.add_request(rid, prompt, sp, kv_transfer_params=ktp)
    out = None
    import time
    for _ in range(20000):
        for o in eng.step():
            if o.request_id == rid and o.finished:
                out = o
        if eng.last_step_empty:
            time.sleep(0.001)
        if out is not None:
            return r, out
    raise AssertionError("request did not finish")


KT = {"kv_connector": "KvxConnector", "kv_role": "kv_both",
      "kv_connector_extra_config": {"transport": "tcp"}}


def test_pd_matches_aggregated():
    P, D, A = make(KT), make(KT), make()
    prompt = np.random.default_rng(0).integers(3, 500, size=150).tolist()
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    _, agg = run(A, "a", prompt, sp)
    agg_r = A.sched  # noqa
    # prefill on P (max_tokens=1), remote decode on D
    rp, op = run(P, "p", prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True),
                 {"do_remote_decode": True})
    ktp = op.kv_transfer_params
    assert ktp and ktp["do_remote_prefill"] and len(ktp["remote_block_ids"]) == 10
    assert P.bm.num_free() < P.bm.num_blocks  # blocks held for the reader
    rd, od = run(D, "d", prompt, sp, ktp)
    assert rd.output_token_ids == A_outputs(A, prompt, sp)
    # D notified P: blocks released on P's next tick
    for _ in range(200):
        P.step()
        if P.bm.num_free() == P.bm.num_blocks:
            break
    assert P.bm.num_free() == P.bm.num_blocks
    assert rd.num_cached_tokens == len(prompt) - 1
    text = D.connector.render_metrics().decode()
    assert "vllm:nixl_xfer_time_seconds_count" in text


def A_outputs(A, prompt, sp):
    return A.generate([prompt], sp)[0].output_token_ids


@pytest.mark.parametrize("policy", ["recompute", "fail"])
def test_pd_load_failure_policy(policy, monkeypatch):
    P = make(KT)
    kt = dict(KT, kv_load_failure_policy=policy)
    D = make(kt)
    prompt = list(range(10, 90))
    _, op = run(P, "p", prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True),
                {"do_remote_decode": True})
    monkeypatch.setenv("LLMD_KVX_FAULT", "drop")
    r, o = run(D, "d", prompt, SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True),
               op.kv_transfer_params)
    if policy == "fail":
        assert o.finish_reason == "error"
    else:
        assert o.finish_reason == "length" and len(r.output_token_ids) == 4
        assert r.num_computed_tokens >= len(prompt)
    assert D.bm.num_free() == D.bm.num_blocks


def test_held_blocks_expire_without_reader():
    kt = dict(KT, kv_connector_extra_config={"transport": "tcp", "abort_timeout": 0.05})
    P = make(kt)
    run(P, "p", list(range(5, 60)), SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True),
        {"do_remote_decode": True})
    assert P.bm.num_free() < P.bm.num_blocks
    import time
    time.sleep(0.1)
    P.step()
    assert P.bm.num_free() == P.bm.num_blocks


def test_prefiller_heartbeat_marks_dead_and_fails_fast(monkeypatch):
    """M13: D pings known prefillers; after 2 misses pulls from that P fail at
    once (recompute policy -> the request still completes locally)."""
    monkeypatch.setenv("LLMD_KVX_HEARTBEAT_S", "0")  # drive heartbeats by hand
    P = make(KT)
    D = make(dict(KT, kv_load_failure_policy="recompute"))
    prompt = list(range(20, 100))
    sp1 = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    _, op = run(P, "p1", prompt, sp1, {"do_remote_decode": True})
    run(D, "d1", prompt, SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True), op.kv_transfer_params)
    ag = D.connector.agent
    key = (op.kv_transfer_params["remote_host"], int(op.kv_transfer_params["remote_port"]))
    assert ag.peer_status()[f"{key[0]}:{key[1]}"] == "alive"
    _, op2 = run(P, "p2", prompt[::-1], sp1, {"do_remote_decode": True})
    P.connector.agent.server.shutdown()          # the prefiller's side channel goes away
    P.connector.agent.server.server_close()
    ag.heartbeat_once()
    assert key not in ag.dead_peers               # one miss is tolerated
    ag.heartbeat_once()
    assert key in ag.dead_peers
    r, o = run(D, "d2", prompt[::-1], SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True),
               op2.kv_transfer_params)
    assert o.finish_reason == "length" and len(r.output_token_ids) == 3   # recomputed locally


def test_abort_during_remote_pull_keeps_blocks_until_done(monkeypatch):
    """aborting a request whose KV pull is in flight must not
    free its destination blocks while the transfer worker can still write them.
    The blocks are released only once the pull reports done, the prefiller is
    told to free its held blocks, and a request admitted meanwhile decodes the
    same tokens as on an aggregated engine."""
    import time

    P = make(KT)
    D = make(KT)
    A = make()
    sp1 = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    prompt = list(range(30, 130))
    other = np.random.default_rng(1).integers(3, 500, size=90).tolist()
    want = A_outputs(A, other, sp)
    _, op = run(P, "p", prompt, sp1, {"do_remote_decode": True})
    assert P.bm.num_free() < P.bm.num_blocks
    monkeypatch.setenv("LLMD_KVX_FAULT", "delay:0.3")
    D.add_request("d", prompt, sp, kv_transfer_params=op.kv_transfer_params)
    D.step()                                    # allocates blocks, starts the (delayed) pull
    assert "d" in D.sched.remote_wait
    held = D.bm.num_blocks - D.bm.num_free()
    assert held > 0
    D.abort("d")
    assert D.bm.num_blocks - D.bm.num_free() == held   # still owned by the in-flight pull
    monkeypatch.delenv("LLMD_KVX_FAULT")
    r2, o2 = run(D, "d2", other, sp)             # admitted while the pull is running
    assert r2.output_token_ids == want
    deadline = time.monotonic() + 10
    while (D.sched.aborted_remote or P.bm.num_free() != P.bm.num_blocks) and time.monotonic() < deadline:
        D.step()
        P.step()
        time.sleep(0.01)
    assert not D.sched.aborted_remote
    assert D.bm.num_free() == D.bm.num_blocks
    assert P.bm.num_free() == P.bm.num_blocks    # abort notif / post-read free reached P
    assert "d" not in D.connector._results


def test_abort_before_pull_starts_notifies_prefiller(monkeypatch):
    """A pull aborted while still queued behind another one is skipped: nothing
    is written locally, P is told to free its held blocks, and D releases the
    destination blocks once the worker reports the skipped job."""
    import time

    monkeypatch.setenv("LLMD_KVX_WORKERS", "1")  # one transfer thread: d2 really waits in the queue
    P = make(KT)
    D = make(KT)
    sp1 = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    _, op1 = run(P, "p1", list(range(40, 120)), sp1, {"do_remote_decode": True})
    _, op2 = run(P, "p2", list(range(140, 220)), sp1, {"do_remote_decode": True})
    monkeypatch.setenv("LLMD_KVX_FAULT", "delay:0.3")
    D.add_request("d1", list(range(40, 120)), SamplingParams(max_tokens=2), kv_transfer_params=op1.kv_transfer_params)
    D.add_request("d2", list(range(140, 220)), SamplingParams(max_tokens=2), kv_transfer_params=op2.kv_transfer_params)
    D.step()                                    # both pulls queued; the worker sleeps in d1's
    assert {"d1", "d2"} <= set(D.sched.remote_wait)
    D.abort("d2")
    monkeypatch.delenv("LLMD_KVX_FAULT")
    deadline = time.monotonic() + 10
    while (D.has_unfinished() or P.bm.num_free() != P.bm.num_blocks) and time.monotonic() < deadline:
        D.step()
        P.step()
        time.sleep(0.01)
    assert P.bm.num_free() == P.bm.num_blocks
    assert D.bm.num_free() == D.bm.num_blocks


def test_pulls_from_different_prefillers_run_concurrently(monkeypatch):
    """N04 (multi-path role): pulls from two prefillers overlap on separate
    transfer workers instead of queueing behind one copy."""
    import time

    P1, P2 = make(KT), make(KT)
    D = make(KT)
    assert D.connector.agent.n_workers >= 2
    sp1 = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    a, b = list(range(10, 90)), list(range(100, 180))
    _, o1 = run(P1, "p1", a, sp1, {"do_remote_decode": True})
    _, o2 = run(P2, "p2", b, sp1, {"do_remote_decode": True})
    monkeypatch.setenv("LLMD_KVX_FAULT", "delay:0.4")
    sp = SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True)
    t0 = time.monotonic()
    D.add_request("d1", a, sp, kv_transfer_params=o1.kv_transfer_params)
    D.add_request("d2", b, sp, kv_transfer_params=o2.kv_transfer_params)
    done = set()
    while len(done) < 2 and time.monotonic() - t0 < 10:
        for o in D.step():
            if o.finished:
                done.add(o.request_id)
        time.sleep(0.002)
    elapsed = time.monotonic() - t0
    assert done == {"d1", "d2"}
    assert elapsed < 0.75, elapsed   # two 0.4 s pulls overlapped (serial would be >= 0.8 s)
    for r in ("d1", "d2"):
        assert D.connector._results.get(r) is None
