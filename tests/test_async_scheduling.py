"""Async scheduling (engine.py _step_async; the reference's
recipes pass vLLM's --async-scheduling, guides/wide-ep-lws/modelserver/gpu/
vllm/base/decode.yaml:89): step N+1 is scheduled and launched before step N's
sampled tokens reach the host, its decode inputs gathered on the device.

Checked against the synchronous engine (async_scheduling=False) on CPU:
identical greedy and seeded-random outputs under chunked prefill, preemption
(a small KV pool), stop tokens (one speculative row discarded), penalties
(forces a settled step), aborts while a step is in flight, and the same number
of streamed outputs per request."""
import numpy as np
import pytest

from llmd_amd.engine.request import SamplingParams
from tests.test_engine import make_engine


def _prompts(seed, lens, vocab=500):
    rng = np.random.default_rng(seed)
    return [rng.integers(3, vocab, size=n).tolist() for n in lens]


def _run(async_on, prompts, params, blocks=64, abort_at=None):
    eng = make_engine(num_gpu_blocks=blocks, async_scheduling=async_on)
    assert eng.async_sched == async_on
    for i, (p, sp) in enumerate(zip(prompts, params)):
        eng.add_request(f"r{i}", p, sp)
    outs = {f"r{i}": [] for i in range(len(prompts))}
    fin = {}
    steps = 0
    while eng.has_unfinished():
        for o in eng.step():
            outs[o.request_id].extend(o.new_token_ids)
            if o.finished:
                fin[o.request_id] = o.finish_reason
        steps += 1
        if abort_at is not None and steps == abort_at:
            eng.abort("r1")
        assert steps < 2000
    return outs, fin


def test_async_matches_sync_greedy_with_chunking_and_preemption():
    prompts = _prompts(1, [5, 90, 200, 33, 64, 17])
    params = [SamplingParams(max_tokens=m, temperature=0.0, ignore_eos=True) for m in (12, 30, 7, 25, 1, 40)]
    a = _run(True, prompts, params, blocks=40)   # 40 x 16 slots: preemptions happen
    s = _run(False, prompts, params, blocks=40)
    assert a == s
    assert all(len(a[0][f"r{i}"]) == params[i].max_tokens for i in range(len(prompts)))


def test_async_matches_sync_seeded_random():
    prompts = _prompts(2, [12, 40, 70])
    params = [SamplingParams(max_tokens=m, temperature=0.8, seed=11 + i, ignore_eos=True)
              for i, m in enumerate((30, 18, 25))]
    assert _run(True, prompts, params) == _run(False, prompts, params)


def test_async_matches_sync_stop_tokens():
    """A stop token is only seen when its step resolves: the async engine has already
    launched one more row for that request, which is discarded. (Greedy: the CPU reference
    sampler draws one random stream per batch, so a batch-composition change would move
    seeded samples there; the GPU sampler is per-row counter-based.)"""
    prompts = _prompts(2, [12, 40, 70])
    base = [SamplingParams(max_tokens=30, temperature=0.0, ignore_eos=True) for _ in range(3)]
    ref, _ = _run(False, prompts, base)
    stops = [[ref[f"r{i}"][10 + 3 * i]] for i in range(3)]
    params = [SamplingParams(max_tokens=30, temperature=0.0, ignore_eos=True, stop_token_ids=st) for st in stops]
    a = _run(True, prompts, params)
    s = _run(False, prompts, params)
    assert a == s
    assert all(a[1][f"r{i}"] == "stop" for i in range(3)), a[1]


def test_async_with_penalties_and_abort():
    prompts = _prompts(3, [20, 30, 25])
    params = [SamplingParams(max_tokens=20, temperature=0.0, ignore_eos=True),
              SamplingParams(max_tokens=40, temperature=0.0, ignore_eos=True),
              SamplingParams(max_tokens=20, temperature=0.0, ignore_eos=True, presence_penalty=1.5,
                             frequency_penalty=0.5)]
    a = _run(True, prompts, params)
    s = _run(False, prompts, params)
    assert a == s
    a2, f2 = _run(True, prompts, params, abort_at=6)
    assert f2.get("r1") in (None, "abort") and len(a2["r1"]) < 40
    assert a2["r0"] == s[0]["r0"] and a2["r2"] == s[0]["r2"]


@pytest.mark.parametrize("async_on", [True, False])
def test_flag_and_engine_args(async_on):
    import argparse

    from llmd_amd.engine.config import add_engine_args, engine_config_from_args

    a = add_engine_args(argparse.ArgumentParser()).parse_args(
        ["--device", "cpu"] + ([] if async_on else ["--no-async-scheduling"]))
    assert engine_config_from_args(a).sched.async_scheduling is async_on


@pytest.mark.gpu
def test_async_matches_sync_on_gpu_with_graphs():
    """On the GPU (hipGraph decode steps, the device-side input gather, per-row seeded
    sampling): greedy and seeded-random outputs identical with async on and off."""
    prompts = _prompts(5, [7, 60, 130, 33, 90])
    params = [SamplingParams(max_tokens=m, temperature=t, seed=3 + i, ignore_eos=True)
              for i, (m, t) in enumerate(((20, 0.0), (35, 0.7), (9, 0.0), (28, 1.0), (40, 0.0)))]

    def run(async_on):
        eng = make_engine(device="cuda", num_gpu_blocks=256, async_scheduling=async_on, enforce_eager=False,
                          cuda_graph_max_bs=8)
        assert eng.async_sched == async_on and eng.runner.graphs
        for i, (p, sp) in enumerate(zip(prompts, params)):
            eng.add_request(f"r{i}", p, sp)
        outs = {f"r{i}": [] for i in range(len(prompts))}
        while eng.has_unfinished():
            for o in eng.step():
                outs[o.request_id].extend(o.new_token_ids)
        return outs

    a, s = run(True), run(False)
    assert a == s
    assert all(len(a[f"r{i}"]) == params[i].max_tokens for i in range(len(prompts)))
