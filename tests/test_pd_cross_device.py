"""P/D token correctness across processes and devices (scripts/pd_check.py;
VERDICT r4 item 2a): a prefill engine hands requests to a decode replica over
the kvx connector and the decoder's greedy tokens must equal an aggregated
engine's on the same weights (the prompt lengths include 143, the hybrid-KV
window boundary case).

* CPU: the harness itself, tcp transport over gloo (hybrid tiny-gpt-oss);
* 1 GPU: P and D share cuda:0 (IPC-mapped pulls, VMM-chunked and plain pools,
  hybrid KV) - the rehearsal form of the cross-device cases;
* >= 2 GPUs: the same across devices, plus the two-sided rccl transport;
* >= 3 GPUs: a TP2 decoder pulling its head slices from a TP1 prefiller.
The reference validates transport and kernel changes in exactly these
topologies (CONTRIBUTING.md:130-140, guides/pd-disaggregation/README.md:336-460).
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NGPU = torch.cuda.device_count() if torch.cuda.is_available() else 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, args, devices=None, env_extra=None, timeout=420):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    if devices is not None:
        env["LLMD_PD_DEVICES"] = devices
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "scripts", "pd_check.py")]
    r = subprocess.run(cmd + args, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith("PDCHECK ")]
    assert r.returncode == 0 and lines, (r.returncode, lines[-1] if lines else r.stdout[-2000:], r.stderr[-2000:])
    d = json.loads(lines[-1][8:])
    assert d["ok"] and d["decoder"]["all_remote"] and d["decoder"]["finished"], d
    return d


def test_pd_check_harness_cpu_tcp_hybrid():
    d = _run(2, ["--device", "cpu", "--transport", "tcp", "--model", "tiny-gpt-oss", "--max-tokens", "6"])
    assert d["exact"] == d["n"]


@pytest.mark.gpu
@pytest.mark.parametrize("model,vmm", [("small-llama", "1"), ("small-llama", "0"), ("tiny-gpt-oss", "1")])
def test_pd_ipc_same_device(model, vmm):
    # TP1 -> TP1 on one device: bit-identical KV; the decoder recomputes the last prompt token in a
    # decode-shaped batch (other GEMM shapes than the aggregated prefill chunk), so an EXACT bf16 logit
    # tie may resolve the other way - _run's ok allows only such ties at a first divergence
    d = _run(2, ["--model", model, "--transport", "ipc"], devices="0,0", env_extra={"LLMD_KV_VMM": vmm})
    assert 2 * d["exact"] >= d["n"] and all(x["near_tie"] for x in d["divergences"]), d


@pytest.mark.gpu
@pytest.mark.skipif(NGPU < 2, reason="needs 2 GPUs")
@pytest.mark.parametrize("model,transport,vmm", [("small-llama", "ipc", "1"), ("small-llama", "ipc", "0"),
                                                 ("tiny-gpt-oss", "ipc", "1"), ("small-llama", "rccl", "1"),
                                                 ("tiny-gpt-oss", "rccl", "1")])
def test_pd_cross_device(model, transport, vmm):
    d = _run(2, ["--model", model, "--transport", transport], devices="0,1", env_extra={"LLMD_KV_VMM": vmm})
    assert 2 * d["exact"] >= d["n"] and all(x["near_tie"] for x in d["divergences"]), d  # see above


@pytest.mark.gpu
@pytest.mark.skipif(NGPU < 3, reason="needs 3 GPUs")
@pytest.mark.parametrize("transport", ["ipc", "rccl"])
def test_pd_tp2_decoder_pulls_head_slices(transport):
    _run(3, ["--model", "small-llama", "--transport", transport, "--decode-tp", "2"], devices="0,1,2")
