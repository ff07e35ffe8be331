"""Wide-EP serving end to end (SURVEY C41 + §2.5 DP/EP; reference
guides/wide-ep-lws/experimental-dp-aware/README.md:1-29 - every DP rank is its
own router endpoint): the single-node launcher starts ONE torchrun group of 2
DP ranks (gloo on CPU) running the OpenAI server with
``--data-parallel-size 2 --enable-expert-parallel``; rank r serves port + r,
experts are sharded over both ranks and exchanged every MoE layer while the
ranks step in lockstep (an idle rank runs dummy forwards). Completions sent to
either rank's port match a single-process engine on the same checkpoint
(greedy, near-tie rule of tests/greedy_check.py)."""
import json
import os
import time
import urllib.request

import numpy as np
import torch

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams
from greedy_check import assert_greedy_match

MODEL = "tiny-gpt-oss"


def _ckpt(path):
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    mc = EngineConfig.create(MODEL, device="cpu").model_config
    torch.manual_seed(0)
    save_safetensors(export_hf(build_model(mc, device="cpu", max_pos=600)), path)


def _post(port, prompt, n):
    body = json.dumps({"model": MODEL, "prompt": prompt, "max_tokens": n, "temperature": 0.0, "ignore_eos": True,
                       "return_token_ids": True}).encode()
    req = urllib.request.Request(f"http://127.0.0.1:{port}/v1/completions", data=body,
                                 headers={"content-type": "application/json"})
    with urllib.request.urlopen(req, timeout=120) as r:
        return json.loads(r.read())["choices"][0]["token_ids"]


def test_wide_ep_dp2_serving_through_launcher(tmp_path):
    from llmd_amd.launch import Launcher, plan

    ck = str(tmp_path / "w.safetensors")
    _ckpt(ck)
    common = ["--load-format", "safetensors", "--weights-path", ck, "--block-size", "16",
              "--num-gpu-blocks-override", "64", "--max-num-seqs", "8", "--max-num-batched-tokens", "64",
              "--max-model-len", "512", "--enforce-eager"]
    topo = {"model": MODEL, "device": "cpu", "master_port_base": 29831,
            "roles": [{"name": "prefill-decode", "replicas": 1, "dp": 2, "port": 18340,
                       "args": common + ["--enable-expert-parallel"]}]}
    specs, doc = plan(topo, str(tmp_path))
    assert [e["port"] for e in doc["endpoints"]] == [18340, 18341]  # one router endpoint per DP rank
    assert sum(bool(s.cmd) for s in specs) == 1 and "--nproc-per-node=2" in specs[0].cmd
    rng = np.random.default_rng(3)
    prompts = [rng.integers(3, 400, size=n).tolist() for n in (37, 12, 70)]
    la = Launcher(topo, workdir=str(tmp_path)).start()
    try:
        ok = la.wait_ready(timeout=300)
        log = open(tmp_path / "prefill-decode-0.log").read()
        assert ok, log[-4000:]
        assert "wide-EP: DP rank 0/2" in log and "wide-EP: DP rank 1/2" in log, log[-4000:]
        got = [None] * len(prompts)
        # rank 0 gets two requests, rank 1 one: the ranks' batches differ and rank 1
        # idles (dummy forwards) while rank 0 still decodes
        import concurrent.futures as cf

        with cf.ThreadPoolExecutor(3) as ex:
            futs = {ex.submit(_post, 18340 + (i == 1), p, 6 if i != 1 else 3): i for i, p in enumerate(prompts)}
            for f in cf.as_completed(futs):
                got[futs[f]] = f.result()
    finally:
        la.stop()
    ref = LLMEngine(EngineConfig.create(MODEL, device="cpu", block_size=16, num_gpu_blocks=64, max_num_seqs=8,
                                        max_num_batched_tokens=64, max_model_len=512, enforce_eager=True,
                                        load_format="safetensors", weights_path=ck))
    want = [r.output_token_ids for r in ref.generate(prompts[:1] + prompts[2:], SamplingParams(
        max_tokens=6, temperature=0.0, ignore_eos=True))]
    want1 = ref.generate(prompts[1:2], SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
    want = [want[0], want1[0].output_token_ids, want[1]]
    assert [len(g) for g in got] == [6, 3, 6]
    assert_greedy_match(ref, prompts, got, want)
