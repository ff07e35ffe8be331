"""Tensor parallelism on CPU (gloo, world 2): TP=2 engine (driver + follower
rank, step-plan broadcast, sharded weights loaded from an HF-format
safetensors checkpoint) must match the TP=1 engine on the same weights."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams
from greedy_check import assert_greedy_match

MODEL = "tiny-llama"


def _cfg(path, model=MODEL, **kw):
    return EngineConfig.create(model, device="cpu", block_size=16, num_gpu_blocks=64, max_num_batched_tokens=64,
                               max_num_seqs=8, max_model_len=512, enforce_eager=True, load_format="safetensors",
                               weights_path=path, **kw)


def _prompts():
    rng = np.random.default_rng(11)
    return [rng.integers(3, 500, size=n).tolist() for n in (37, 90, 5)]


def _worker(rank, world, port, path, out, model=MODEL):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from llmd_amd.parallel.state import destroy, init_distributed

    init_distributed(tp_size=world, backend="gloo")
    cfg = _cfg(path, model, tensor_parallel_size=world)
    if rank == 0:
        eng = LLMEngine(cfg)
        reqs = eng.generate(_prompts(), SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True,
                                                       logprobs=1))
        eng.shutdown()
        torch.save({"tokens": [r.output_token_ids for r in reqs],
                    "lp": [r.output_logprobs for r in reqs]}, out)
    else:
        from llmd_amd.engine.tp_worker import run_follower

        run_follower(cfg)
    destroy()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("model", [MODEL, "tiny-opt"])
def test_tp2_matches_tp1(tmp_path, model):
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    path = str(tmp_path / "model.safetensors")
    cfg1 = _cfg(None, model)
    torch.manual_seed(0)  # fixed weights: TP sums in another order, so a random model can hold near-ties
    m = build_model(cfg1.model_config, device="cpu", max_pos=600)
    for n, prm in m.named_parameters():  # non-zero biases (OPT): sharded / replicated biases must be placed right
        if n.endswith("bias"):
            torch.nn.init.normal_(prm, std=0.05)
    save_safetensors(export_hf(m), path)
    eng = LLMEngine(_cfg(path, model))
    ref = eng.generate(_prompts(), SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True, logprobs=1))
    out = str(tmp_path / "tp2.pt")
    mp.spawn(_worker, args=(2, _free_port(), path, out, model), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    # TP all-reduces sum the row-parallel shards in another order (bf16): a
    # first divergence must be a near-tie of the TP1 engine (greedy_check)
    assert_greedy_match(eng, _prompts(), got["tokens"], [r.output_token_ids for r in ref])
    for r, toks, lps in zip(ref, got["tokens"], got["lp"]):
        if toks == r.output_token_ids:
            assert np.allclose(lps, r.output_logprobs, atol=0.05)


def _pd_worker(rank, world, port, path, out):
    """rank 0: TP1 prefiller (kv_producer); ranks 1, 2: one TP2 decode replica
    (kv_consumer) whose driver schedules and whose follower pulls its own
    KV-head slice (kvx TP re-slicing, TCP transport on CPU)."""
    import torch.distributed as dist

    from llmd_amd.parallel.state import ParallelState, set_state

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tg = dist.new_group([1, 2])
    kt = {"kv_connector": "KvxConnector", "kv_role": "kv_producer" if rank == 0 else "kv_consumer",
          "kv_connector_extra_config": {"transport": "tcp"}}
    if rank > 0:
        set_state(ParallelState(world_size=world, rank=rank, tp_size=2, tp_rank=rank - 1, tp_group=tg,
                                tp_cpu_group=tg, cpu_group=tg, backend="gloo", tp_src=1))
    cfg = _cfg(path, kv_transfer_config=kt)
    box = [None]
    if rank == 0:
        eng = LLMEngine(cfg)
        params = []
        for i, p in enumerate(_prompts()):
            eng.add_request(f"p{i}", p, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True),
                            kv_transfer_params={"do_remote_decode": True})
        done = {}
        while len(done) < len(_prompts()):
            for o in eng.step():
                if o.finished:
                    done[o.request_id] = o.kv_transfer_params
        box = [[done[f"p{i}"] for i in range(len(_prompts()))]]
        dist.broadcast_object_list(box, src=0)
        held = len(eng.connector.agent.held)
        dist.barrier()  # decoders finished
        for _ in range(100):  # both decode ranks sent their free: blocks come back
            eng.step()
        torch.save({"held_before": held, "held_after": len(eng.connector.agent.held),
                    "free": eng.bm.num_free(), "total": eng.bm.num_blocks}, out + ".p")
        eng.connector.close()
    elif rank == 1:
        eng = LLMEngine(cfg)
        dist.broadcast_object_list(box, src=0)
        reqs = [eng.add_request(f"d{i}", p, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True),
                                kv_transfer_params=box[0][i]) for i, p in enumerate(_prompts())]
        import time

        while eng.has_unfinished():
            eng.step()
            if eng.last_step_empty:
                time.sleep(0.001)
        torch.save({"tokens": [r.output_token_ids for r in reqs],
                    "cached": [r.num_cached_tokens for r in reqs]}, out)
        eng.shutdown()
        dist.barrier()
    else:
        from llmd_amd.engine.tp_worker import run_follower

        # the driver's engine start-up is collective with this runner's: receive
        # the params only once both are built
        run_follower(cfg, on_ready=lambda: dist.broadcast_object_list(box, src=0))
        dist.barrier()
    dist.destroy_process_group()


def test_pd_tp1_prefill_to_tp2_decode(tmp_path):
    """A TP1 prefiller feeding a TP2 decode replica (the reference's P/D
    shape, decoders TP>1) produces the aggregated TP1 engine's tokens: every
    decode rank must have pulled its own KV-head slice, and the prefiller
    frees its blocks only after both ranks read them."""
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    path = str(tmp_path / "model.safetensors")
    torch.manual_seed(0)
    save_safetensors(export_hf(build_model(_cfg(None).model_config, device="cpu", max_pos=600)), path)
    ref_eng = LLMEngine(_cfg(path))
    ref = ref_eng.generate(_prompts(), SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))
    out = str(tmp_path / "pd.pt")
    mp.spawn(_pd_worker, args=(3, _free_port(), path, out), nprocs=3, join=True)
    got = torch.load(out, weights_only=True)
    assert_greedy_match(ref_eng, _prompts(), got["tokens"], [r.output_token_ids for r in ref])
    for cached, p in zip(got["cached"], _prompts()):
        assert cached == len(p) - 1  # prompt KV came over kvx, not recomputed
    pg = torch.load(out + ".p", weights_only=True)
    assert pg["held_before"] == 3 and pg["held_after"] == 0 and pg["free"] == pg["total"]
