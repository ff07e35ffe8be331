"""RL weight sync and sleep / wake-up (engine/weight_sync.py).

* update_from_disk: an engine built on checkpoint B and updated from
  checkpoint A generates exactly what an engine built on A does (bf16 and
  online fp8 W8A8, whose re-quantisation must equal quantising at load).
* update_from_group: a trainer process broadcasts A's tensors over a
  stand-alone gloo group to a TP=2 engine (driver + follower); the updated
  engine matches a TP=1 engine built on A (greedy_check near-tie rule).
* HTTP: /update_weights_from_disk, /sleep, /is_sleeping, /wake_up.
* GPU: sleep releases the weights and KV pool, wake-up restores them and
  re-captures the decode hipGraphs; outputs are unchanged.
"""
import asyncio
import os
import socket

import aiohttp
import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
from aiohttp import web

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams
from greedy_check import assert_greedy_match

MODEL = "tiny-llama"
SP = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True, logprobs=1)


def _cfg(path, device="cpu", model=MODEL, **kw):
    kw.setdefault("enforce_eager", device == "cpu")
    return EngineConfig.create(model, device=device, block_size=16, num_gpu_blocks=64, max_num_batched_tokens=64,
                               max_num_seqs=8, max_model_len=512, load_format="safetensors", weights_path=path, **kw)


def _prompts():
    rng = np.random.default_rng(5)
    return [rng.integers(3, 500, size=n).tolist() for n in (41, 77, 9)]


def _ckpts(tmp_path, tags=("a", "b"), model=MODEL):
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    mc = _cfg(None, model=model).model_config
    paths = []
    for seed, tag in enumerate(tags):
        torch.manual_seed(seed)
        p = str(tmp_path / f"{tag}.safetensors")
        save_safetensors(export_hf(build_model(mc, device="cpu", max_pos=600)), p)
        paths.append(p)
    return paths


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(eng):
    return [(r.output_token_ids, r.output_logprobs) for r in eng.generate(_prompts(), SP)]


@pytest.mark.parametrize("model,quant", [(MODEL, None), (MODEL, "fp8"), ("tiny-gpt-oss", "mxfp4")])
def test_update_from_disk_matches_fresh_engine(tmp_path, model, quant):
    """mxfp4: the MXFP4 experts are re-quantised from the update exactly as at load."""
    a, b = _ckpts(tmp_path, model=model)
    ref = _run(LLMEngine(_cfg(a, model=model, quantization=quant)))
    eng = LLMEngine(_cfg(b, model=model, quantization=quant))
    before = _run(eng)
    assert [t for t, _ in before] != [t for t, _ in ref]  # the two checkpoints really differ
    res = eng.weight_sync_cmd({"op": "update_from_disk", "path": a})
    assert res["updated"] == len(eng.runner.model.weight_specs()) and res["version"] == 1
    assert _run(eng) == ref


def _tp_worker(rank, world, port, ws_port, a, b, out):
    """rank 0: trainer (WeightSender); ranks 1, 2: TP=2 engine (driver, follower)."""
    from safetensors.torch import load_file

    from llmd_amd.engine.weight_sync import WeightSender

    tensors = load_file(a)
    metas = WeightSender.metas(tensors)
    if rank == 0:
        snd = WeightSender("127.0.0.1", ws_port, world_size=3).connect()
        snd.send(tensors)
        return
    er = rank - 1
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(er), WORLD_SIZE="2",
                      LOCAL_RANK=str(er))
    from llmd_amd.parallel.state import destroy, init_distributed

    init_distributed(tp_size=2, backend="gloo")
    cfg = _cfg(b, tensor_parallel_size=2)
    if er == 0:
        eng = LLMEngine(cfg)
        eng.weight_sync_cmd({"op": "init_group", "addr": "127.0.0.1", "port": ws_port, "rank_offset": 1,
                             "world_size": 3, "backend": "gloo"})
        res = eng.weight_sync_cmd({"op": "update_from_group", "metas": metas})
        reqs = eng.generate(_prompts(), SP)
        eng.shutdown()
        torch.save({"tokens": [r.output_token_ids for r in reqs], "updated": res["updated"]}, out)
    else:
        from llmd_amd.engine.tp_worker import run_follower

        run_follower(cfg)
    destroy()


def test_update_from_trainer_group_tp2(tmp_path):
    a, b = _ckpts(tmp_path)
    eng_a = LLMEngine(_cfg(a))
    ref = [r.output_token_ids for r in eng_a.generate(_prompts(), SP)]
    out = str(tmp_path / "tp2.pt")
    mp.spawn(_tp_worker, args=(3, _free_port(), _free_port(), a, b, out), nprocs=3, join=True)
    got = torch.load(out, weights_only=True)
    assert got["updated"] == len(eng_a.runner.model.weight_specs())
    assert_greedy_match(eng_a, _prompts(), got["tokens"], ref)


async def _serve(app):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


def test_http_weight_update_and_sleep(tmp_path):
    from llmd_amd.serving.api_server import build_server

    a, b = _ckpts(tmp_path)
    ref = [r.output_token_ids for r in LLMEngine(_cfg(a)).generate(_prompts()[:1], SP)]
    body = {"model": MODEL, "prompt": _prompts()[0], "max_tokens": 6, "temperature": 0.0, "ignore_eos": True,
            "return_token_ids": True}

    async def main():
        srv = build_server(_cfg(b))
        r1, port = await _serve(srv.app())
        base = f"http://127.0.0.1:{port}"
        res = {}
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(base + "/update_weights_from_disk", json={"path": a}) as r:
                    res["upd"] = (r.status, await r.json())
                async with s.post(base + "/update_weights_from_disk", json={"path": str(tmp_path / "nope")}) as r:
                    res["bad"] = r.status
                async with s.post(base + "/v1/completions", json=body) as r:
                    res["toks"] = (await r.json())["choices"][0]["token_ids"]
                async with s.post(base + "/sleep", json={"level": 1}) as r:
                    res["sleep"] = (r.status, await r.json())
                async with s.get(base + "/is_sleeping") as r:
                    res["is1"] = await r.json()
                async with s.post(base + "/update_weights_from_disk", json={"path": a}) as r:
                    res["upd_asleep"] = r.status  # refused while asleep
                async with s.post(base + "/wake_up") as r:
                    res["wake"] = r.status
                async with s.get(base + "/is_sleeping") as r:
                    res["is0"] = await r.json()
                async with s.post(base + "/v1/completions", json=body) as r:
                    res["toks2"] = (await r.json())["choices"][0]["token_ids"]
        finally:
            await r1.cleanup()
            srv.aeng.shutdown()
        return res

    res = asyncio.run(main())
    assert res["upd"][0] == 200 and res["upd"][1]["updated"] > 0
    assert res["bad"] == 400
    assert res["toks"] == ref[0] and res["toks2"] == ref[0]
    assert res["sleep"][0] == 200 and res["is1"] == {"is_sleeping": True, "level": 1, "weights_pending": False}
    assert res["upd_asleep"] == 409
    assert res["wake"] == 200 and res["is0"]["is_sleeping"] is False


@pytest.mark.gpu
def test_sleep_wake_gpu_releases_memory_and_recaptures(tmp_path):
    a, b = _ckpts(tmp_path)
    ref = _run(LLMEngine(_cfg(a, device="cuda")))
    eng = LLMEngine(_cfg(b, device="cuda"))
    assert eng.runner.graphs, "decode hipGraphs must be captured for this test"
    torch.cuda.synchronize()
    used0 = torch.cuda.memory_allocated()
    res = eng.weight_sync_cmd({"op": "sleep", "level": 1})
    used1 = torch.cuda.memory_allocated()
    assert used0 - used1 >= 0.9 * res["freed_bytes"] > 0, (used0, used1, res)
    eng.weight_sync_cmd({"op": "wake_up"})
    assert eng.runner.graphs
    eng.weight_sync_cmd({"op": "update_from_disk", "path": a})
    got = _run(eng)
    assert [t for t, _ in got] == [t for t, _ in ref]
    # level 2 drops the weights: the trainer (here: the checkpoint) restores them after wake-up
    eng.weight_sync_cmd({"op": "sleep", "level": 2})
    eng.weight_sync_cmd({"op": "wake_up"})
    eng.weight_sync_cmd({"op": "update_from_disk", "path": a})
    assert [t for t, _ in _run(eng)] == [t for t, _ in ref]


@pytest.mark.gpu
def test_sleep_with_kv_offload_gpu_releases_pool(tmp_path):
    """With the host KV tier configured the offloader also references the pool
    (and staging copies of it): sleep must release it all the same."""
    a, _ = _ckpts(tmp_path)
    off = {"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}
    ref = _run(LLMEngine(_cfg(a, device="cuda")))
    eng = LLMEngine(_cfg(a, device="cuda", kv_offload_config=off))
    assert _run(eng) == ref
    assert eng.offload.pending or eng.offload.stats["offloaded"] > 0
    torch.cuda.synchronize()
    kv_bytes = eng.runner.kv.untyped_storage().nbytes()
    used0 = torch.cuda.memory_allocated()
    res = eng.weight_sync_cmd({"op": "sleep", "level": 1})
    used1 = torch.cuda.memory_allocated()
    assert eng.offload.kv is None and not eng.offload.pending
    assert used0 - used1 >= 0.9 * res["freed_bytes"] > kv_bytes, (used0, used1, res, kv_bytes)
    eng.weight_sync_cmd({"op": "wake_up"})
    assert eng.offload.kv is eng.runner.kv
    # after wake-up the prompts' prefixes come back from the host tier, so only their
    # tails are recomputed: same tokens, logprobs equal up to the GEMM path chosen for
    # the smaller prefill batch (ops.linear autotunes per M bucket)
    got = _run(eng)
    assert [t for t, _ in got] == [t for t, _ in ref]
    for (_, lp), (_, lr) in zip(got, ref):
        assert np.allclose(lp, lr, atol=2e-3), (lp, lr)


@pytest.mark.gpu
def test_update_from_disk_fp8_gpu(tmp_path):
    a, b = _ckpts(tmp_path)
    ref = _run(LLMEngine(_cfg(a, device="cuda", quantization="fp8")))
    eng = LLMEngine(_cfg(b, device="cuda", quantization="fp8"))
    eng.weight_sync_cmd({"op": "update_from_disk", "path": a})
    assert [t for t, _ in _run(eng)] == [t for t, _ in ref]


def test_update_invalidates_offloaded_kv(tmp_path):
    """Host / FS KV tiers hold KV of the old weights: after an update a request
    with the same prefix must recompute it, not reload it."""
    a, b = _ckpts(tmp_path)
    ref = _run(LLMEngine(_cfg(a)))
    eng = LLMEngine(_cfg(b, kv_offload_config={"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}))
    _run(eng)
    off = eng.offload
    off.poll()
    assert off.stats["offloaded"] > 0 and off.slot_of
    ns0 = off.ns
    eng.weight_sync_cmd({"op": "update_from_disk", "path": a})
    assert not off.slot_of and off.weights_id == eng.weight_sync.weights_id and off.ns != ns0
    assert [e[0] for e in off.take_events()].count(1) > 0  # host-tier removals reach the router's index
    loaded = (off.stats["loaded_cpu"], off.stats["loaded_fs"])
    assert _run(eng) == ref
    assert (off.stats["loaded_cpu"], off.stats["loaded_fs"]) == loaded


def test_level2_wake_holds_requests_until_weights_arrive(tmp_path):
    """After a level-2 sleep the weights are uninitialised storage until the
    trainer sends them: a request queued meanwhile must not be served by the
    woken engine before the update."""
    a, _ = _ckpts(tmp_path)
    ref = _run(LLMEngine(_cfg(a)))
    eng = LLMEngine(_cfg(a))
    eng.weight_sync_cmd({"op": "sleep", "level": 2})
    reqs = [eng.add_request(f"q{i}", p, SP) for i, p in enumerate(_prompts())]
    assert eng.step() == []
    res = eng.weight_sync_cmd({"op": "wake_up"})
    assert res["weights_pending"] and eng.weights_pending
    for _ in range(5):
        assert eng.step() == []
    assert all(not r.output_token_ids for r in reqs)
    eng.weight_sync_cmd({"op": "update_from_disk", "path": a})
    assert not eng.weights_pending
    while eng.has_unfinished():
        eng.step()
    assert [(r.output_token_ids, r.output_logprobs) for r in reqs] == ref


def test_level2_wake_holds_http_requests(tmp_path):
    """The same through the HTTP server: a completion sent while asleep (level
    2) is answered only after /update_weights_from_disk, with the new weights'
    tokens."""
    from llmd_amd.serving.api_server import build_server

    a, _ = _ckpts(tmp_path)
    ref = _run(LLMEngine(_cfg(a)))
    body = {"model": MODEL, "prompt": _prompts()[0], "max_tokens": 6, "temperature": 0.0,
            "ignore_eos": True, "return_token_ids": True}

    async def main():
        srv = build_server(_cfg(a))
        r1, port = await _serve(srv.app())
        base = f"http://127.0.0.1:{port}"
        res = {}
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(base + "/sleep", json={"level": 2}) as r:
                    res["sleep"] = r.status
                task = asyncio.ensure_future(s.post(base + "/v1/completions", json=body))
                await asyncio.sleep(0.3)
                async with s.post(base + "/wake_up") as r:
                    res["wake"] = (r.status, await r.json())
                async with s.get(base + "/is_sleeping") as r:
                    res["pending"] = (await r.json())["weights_pending"]
                await asyncio.sleep(0.5)
                res["served_early"] = task.done()
                async with s.post(base + "/update_weights_from_disk", json={"path": a}) as r:
                    res["upd"] = r.status
                resp = await asyncio.wait_for(task, 30)
                res["toks"] = (await resp.json())["choices"][0]["token_ids"]
                resp.release()
        finally:
            await r1.cleanup()
            srv.aeng.shutdown()
        return res

    res = asyncio.run(main())
    assert res["sleep"] == 200 and res["wake"][0] == 200 and res["wake"][1]["weights_pending"]
    assert res["pending"] is True and res["served_early"] is False
    assert res["upd"] == 200 and res["toks"] == ref[0][0]


def test_fs_kv_namespace_survives_restart(tmp_path):
    """FS-tier keys are namespaced by a stable identity of the weights, not by a
    per-process update counter: an engine restarted on the same fs_root that
    goes through a DIFFERENT update must not reload the first process's KV,
    while an engine started from the checkpoint that KV was computed with
    reloads it."""
    a, b, c = _ckpts(tmp_path, ("a", "b", "c"))
    off = {"cpu_bytes_to_use": 64 << 20, "fs_root": str(tmp_path / "kv")}
    ref_a, ref_c = _run(LLMEngine(_cfg(a))), _run(LLMEngine(_cfg(c)))
    e1 = LLMEngine(_cfg(b, kv_offload_config=off))
    e1.weight_sync_cmd({"op": "update_from_disk", "path": a})
    assert _run(e1) == ref_a
    e1.offload.poll()
    assert e1.offload.stats["offloaded"] > 0
    e1.offload.fs.flush()
    # restart: same initial weights, then a different update (the old counter-based
    # scheme reused namespace "w1" here and reloaded KV computed with A)
    e2 = LLMEngine(_cfg(b, kv_offload_config=off))
    e2.weight_sync_cmd({"op": "update_from_disk", "path": c})
    assert _run(e2) == ref_c
    assert e2.offload.stats["loaded_fs"] == 0
    # a replica started from A shares the namespace of e1's post-update KV
    e3 = LLMEngine(_cfg(a, kv_offload_config=off))
    e3.offload.slot_of.clear()
    assert _run(e3) == ref_a
    assert e3.offload.stats["loaded_fs"] > 0
    # trainer-named versions: the same name is the same namespace in any process
    e4 = LLMEngine(_cfg(b, kv_offload_config=off))
    e4.weight_sync_cmd({"op": "update_from_disk", "path": a, "weights_version": "step-7"})
    e5 = LLMEngine(_cfg(c, kv_offload_config=off))
    e5.weight_sync_cmd({"op": "update_from_disk", "path": a, "weights_version": "step-7"})
    assert e4.offload.ns == e5.offload.ns != e1.offload.ns
