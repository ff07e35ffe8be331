"""Wide-EP on CPU (gloo, world 2): DP attention + EP MoE in lockstep. Each DP
rank serves its own requests (one rank finishes early and keeps stepping with
dummy forwards), experts are sharded over both ranks and exchanged with either
all2all backend; every rank's greedy outputs must equal a single-process
engine on the same weights."""
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

PROMPTS = {0: [41, 97, 8], 1: [13, 66]}
NTOK = {0: 6, 1: 3}


def _cfg(model, path, **kw):
    return EngineConfig.create(model, device="cpu", block_size=16, num_gpu_blocks=64, max_num_batched_tokens=64,
                               max_num_seqs=8, max_model_len=512, enforce_eager=True, load_format="safetensors",
                               weights_path=path, **kw)


def _prompts(rank):
    rng = np.random.default_rng(100 + rank)
    return [rng.integers(3, 500, size=n).tolist() for n in PROMPTS[rank]]


def _worker(rank, world, port, model, path, backend, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from llmd_amd.parallel.state import destroy, init_distributed

    init_distributed(tp_size=1, backend="gloo")
    eng = LLMEngine(_cfg(model, path, data_parallel_size=world, enable_expert_parallel=True,
                         all2all_backend=backend))
    assert eng.dp_lockstep
    sp = SamplingParams(max_tokens=NTOK[rank], temperature=0.0, ignore_eos=True)
    reqs = [eng.add_request(f"r{rank}-{i}", p, sp) for i, p in enumerate(_prompts(rank))]
    steps = 0
    while eng.dp_has_unfinished():
        eng.step()
        steps += 1
    torch.save({"tokens": [r.output_token_ids for r in reqs], "steps": steps}, f"{out}.{rank}")
    destroy()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("model", ["tiny-deepseek", "tiny-gpt-oss"])
@pytest.mark.parametrize("backend", ["allgather_reducescatter", "alltoall"])
def test_dp_ep_lockstep_matches_single_process(tmp_path, model, backend):
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    path = str(tmp_path / "w.safetensors")
    if not os.path.exists(path):
        cfg = _cfg(model, None)
        save_safetensors(export_hf(build_model(cfg.model_config, device="cpu", max_pos=600)), path)
    ref = LLMEngine(_cfg(model, path))
    want = {}
    for rank in (0, 1):
        sp = SamplingParams(max_tokens=NTOK[rank], temperature=0.0, ignore_eos=True)
        want[rank] = [r.output_token_ids for r in ref.generate(_prompts(rank), sp)]
    out = str(tmp_path / "ep")
    mp.spawn(_worker, args=(2, _free_port(), model, path, backend, out), nprocs=2, join=True)
    for rank in (0, 1):
        got = torch.load(f"{out}.{rank}", weights_only=True)["tokens"]
        # EP combines expert partial sums in another order (bf16): greedy_check
        assert_greedy_match(ref, _prompts(rank), got, want[rank])
    # the early-finishing rank kept stepping (dummy forwards) until rank 0 was done
    assert torch.load(f"{out}.1", weights_only=True)["steps"] == torch.load(f"{out}.0", weights_only=True)["steps"]
