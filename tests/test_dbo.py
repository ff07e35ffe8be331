"""Dual-batch overlap on CPU, world 2 (gloo): decode steps (and
steps with prefill chunks above --dbo-prefill-token-threshold) split into two
micro-batches whose layers alternate (two HIP streams on GPU, each
with its own EP channel); greedy outputs still match a single-process engine,
including the early-finishing rank that keeps stepping with dummy halves."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams

from greedy_check import assert_greedy_match
from test_wide_ep import NTOK, _cfg, _free_port, _prompts


def _worker(rank, world, port, model, path, backend, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from llmd_amd.parallel.state import destroy, init_distributed

    init_distributed(tp_size=1, backend="gloo")
    eng = LLMEngine(_cfg(model, path, data_parallel_size=world, enable_expert_parallel=True,
                         all2all_backend=backend, enable_dbo=True, dbo_decode_token_threshold=1))
    calls = {"n": 0, "p": 0}
    orig = eng.runner.execute_dbo

    def counted(so, *a, **k):
        calls["n"] += 1
        calls["p"] += int(so is not None and bool(so.prefills))
        return orig(so, *a, **k)

    eng.runner.execute_dbo = counted
    sp = SamplingParams(max_tokens=NTOK[rank], temperature=0.0, ignore_eos=True)
    reqs = [eng.add_request(f"r{rank}-{i}", p, sp) for i, p in enumerate(_prompts(rank))]
    while eng.dp_has_unfinished():
        eng.step()
    torch.save({"tokens": [r.output_token_ids for r in reqs], "dbo_steps": calls["n"],
                "dbo_prefill_steps": calls["p"]}, f"{out}.{rank}")
    destroy()


@pytest.mark.parametrize("backend", ["allgather_reducescatter", "alltoall"])
def test_dbo_world2_matches_single_process(tmp_path, backend):
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    model = "tiny-gpt-oss"
    path = str(tmp_path / "w.safetensors")
    save_safetensors(export_hf(build_model(_cfg(model, None).model_config, device="cpu", max_pos=600)), path)
    ref = LLMEngine(_cfg(model, path))
    want = {}
    for rank in (0, 1):
        sp = SamplingParams(max_tokens=NTOK[rank], temperature=0.0, ignore_eos=True)
        want[rank] = [r.output_token_ids for r in ref.generate(_prompts(rank), sp)]
    out = str(tmp_path / "dbo")
    mp.spawn(_worker, args=(2, _free_port(), model, path, backend, out), nprocs=2, join=True)
    for rank in (0, 1):
        d = torch.load(f"{out}.{rank}", weights_only=True)
        assert d["dbo_steps"] >= 3 and d["dbo_prefill_steps"] >= 1
        assert_greedy_match(ref, _prompts(rank), d["tokens"], want[rank])
