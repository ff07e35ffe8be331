"""Cross-device paths of the N > 1 topologies (bench.py / launch.py), on real GPUs.

* every pre-flight check (llmd_amd/parallel/preflight.py: peer access, IPC and
  VMM pulls, symm all-reduce vs RCCL, symm EP vs the RCCL all_to_all path)
  with one process per physical GPU - skipped below 2 devices;
* the same IPC / VMM / symm-all-reduce checks with two ranks sharing cuda:0
  (the 1-GPU rehearsal: the kernels still go through IPC-mapped memory);
* a TP2 decode replica (two GPUs) produces TP1's greedy tokens - skipped below
  2 devices.
Each case runs its ranks as subprocesses with their own timeout so a hang
fails the test instead of the suite."""
import json
import os
import subprocess
import sys
import textwrap

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NGPU = torch.cuda.device_count() if torch.cuda.is_available() else 0

_RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, datetime
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    rank, world = int(sys.argv[1]), int(sys.argv[2])
    dev = int(sys.argv[3]) if sys.argv[3] != "rank" else rank
    checks = sys.argv[4].split(",")
    torch.cuda.set_device(dev)
    backend = sys.argv[5]
    kw = {{"device_id": torch.device("cuda", dev)}} if backend == "nccl" else {{}}
    dist.init_process_group(backend, init_method="tcp://127.0.0.1:" + sys.argv[6], rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=120), **kw)
    from llmd_amd.parallel import preflight
    out = preflight.run(rank, world, torch.device("cuda", dev), checks=checks, raise_on_fail=False,
                        log=lambda m: None)
    if rank == 0:
        print("RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
""")


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(world, dev, checks, backend, timeout=240):
    script = _RANK_SCRIPT.format(root=ROOT)
    port = str(_free_port())
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    procs = [subprocess.Popen([sys.executable, "-c", script, str(r), str(world), dev, ",".join(checks), backend,
                               port], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), "\n---\n".join(outs)
    line = next(l for l in outs[0].splitlines() if l.startswith("RESULT "))
    return json.loads(line[7:])


def test_preflight_two_ranks_one_gpu():
    """1-GPU rehearsal: IPC + VMM pulls and the symm all-reduce (vs gloo's sum, bit for bit)."""
    res = _run_ranks(2, "0", ["ipc", "vmm", "symm_ar"], "gloo")
    for k in ("ipc", "vmm", "symm_ar"):
        assert res["preflight"][k]["ok"], (k, res["preflight"][k])


@pytest.mark.skipif(NGPU < 2, reason="needs 2 GPUs")
def test_preflight_two_gpus():
    res = _run_ranks(2, "rank", list(("peer", "ipc", "vmm", "symm_ar", "ep")), "nccl")
    for k, v in res["preflight"].items():
        assert v["ok"], (k, v)


@pytest.mark.skipif(NGPU < 8, reason="needs 8 GPUs")
def test_preflight_eight_gpus():
    res = _run_ranks(8, "rank", ["peer", "ipc", "vmm", "symm_ar", "ep"], "nccl", timeout=400)
    for k, v in res["preflight"].items():
        assert v["ok"], (k, v)


_TP_SCRIPT = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, {root!r})
    import torch
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    from llmd_amd.parallel.state import init_distributed
    init_distributed(tp_size=world)
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams
    cfg = EngineConfig.create("small-llama", device="cuda", block_size=64, num_gpu_blocks=64,
                              max_num_batched_tokens=512, max_num_seqs=4, max_model_len=1024,
                              tensor_parallel_size=world, load_format="safetensors", weights_path={path!r})
    if rank == 0:
        eng = LLMEngine(cfg)
        reqs = eng.generate({prompts!r}, SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))
        print("TOKENS " + json.dumps([r.output_token_ids for r in reqs]), flush=True)
        eng.shutdown()
    else:
        from llmd_amd.engine.tp_worker import run_follower
        run_follower(cfg)
""")


@pytest.mark.skipif(NGPU < 2, reason="needs 2 GPUs")
def test_tp2_decode_matches_tp1_greedy(tmp_path):
    """A TP2 replica on two GPUs (RCCL / custom all-reduce over xGMI, hipGraph
    decode) generates the TP1 greedy tokens of the same checkpoint (a first
    divergence must be a near-tie of the TP1 engine: greedy_check)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from greedy_check import assert_greedy_match

    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, save_safetensors

    path = str(tmp_path / "model.safetensors")
    kw = dict(block_size=64, num_gpu_blocks=64, max_num_batched_tokens=512, max_num_seqs=4, max_model_len=1024)
    torch.manual_seed(0)
    m = build_model(EngineConfig.create("small-llama", device="cpu", **kw).model_config, device="cpu", max_pos=1100)
    save_safetensors(export_hf(m), path)
    del m
    prompts = [list(range(10, 200)), [7] * 77]
    port = str(_free_port())
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port, WORLD_SIZE="2")
    script = _TP_SCRIPT.format(root=ROOT, path=path, prompts=prompts)
    procs = [subprocess.Popen([sys.executable, "-c", script], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    try:
        outs = [p.communicate(timeout=300)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), "\n---\n".join(outs)
    got = json.loads(next(l for l in outs[0].splitlines() if l.startswith("TOKENS "))[7:])
    eng = LLMEngine(EngineConfig.create("small-llama", device="cuda", load_format="safetensors", weights_path=path,
                                        **kw))
    ref = eng.generate(prompts, SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))
    assert_greedy_match(eng, prompts, got, [r.output_token_ids for r in ref])
