"""Tensor parallelism on CPU (gloo, world 2): TP=2 engine (driver + follower
rank, step-plan broadcast, sharded weights loaded from an HF-format
safetensors checkpoint) must match the TP=1 engine on the same weights."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams

MODEL = "tiny-llama"


def _cfg(path, **kw):
    return EngineConfig.create(MODEL, device="cpu", block_size=16, num_gpu_blocks=64, max_num_batched_tokens=64,
                               max_num_seqs=8, max_model_len=512, enforce_eager=True, load_format="safetensors",
                               weights_path=path, **kw)


def _prompts():
    rng = np.random.default_rng(11)
    return [rng.integers(3, 500, size=n).tolist() for n in (37, 90, 5)]


def _worker(rank, world, port, path, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from llmd_amd.parallel.state import destroy, init_distributed

    init_distributed(tp_size=world, backend="gloo")
    cfg = _cfg(path, tensor_parallel_size=world)
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


def test_tp2_matches_tp1(tmp_path):
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    path = str(tmp_path / "model.safetensors")
    cfg1 = _cfg(None)
    save_safetensors(export_hf(build_model(cfg1.model_config, device="cpu", max_pos=600)), path)
    eng = LLMEngine(_cfg(path))
    ref = eng.generate(_prompts(), SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True, logprobs=1))
    out = str(tmp_path / "tp2.pt")
    mp.spawn(_worker, args=(2, _free_port(), path, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    for r, toks, lps in zip(ref, got["tokens"], got["lp"]):
        assert toks == r.output_token_ids
        assert np.allclose(lps, r.output_logprobs, atol=0.05)
