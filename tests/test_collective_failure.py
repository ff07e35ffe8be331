"""Fail-loud collectives (the reference runs NCCL under a
watchdog, TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC=15, docker/Dockerfile.cuda:607-608).

A symm barrier that times out sets a host-mapped failure word
(csrc/ops/symm.hip, llmd_symm_host_err). Here:
* CPU: with the word set, ``LLMEngine.step`` raises CollectiveFailure before
  any token of that step is emitted; the serving loop exits the process with
  status 70 (a restart of the replica is the only recovery);
* GPU (2 processes on one device): a peer that never enters the all-reduce
  makes rank 0's kernel time out, set the word, and ``check_health`` raise.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from llmd_amd.engine.request import SamplingParams
from llmd_amd.parallel import symm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def fake_word(monkeypatch):
    w = ctypes.c_uint32(0)
    monkeypatch.setattr(symm, "_herr_word", w)
    return w


def test_engine_step_raises_before_emitting(fake_word):
    from tests.test_engine import make_engine

    eng = make_engine(async_scheduling=False)
    prompt = np.random.default_rng(1).integers(3, 500, size=40).tolist()
    eng.add_request("a", prompt, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
    outs = eng.step()  # healthy: the prefill step emits the first token
    assert [o.request_id for o in outs] == ["a"]
    n_tok = len(eng.sched.requests["a"].output_token_ids)
    fake_word.value = 1  # a symm kernel of this process timed out during the next step
    with pytest.raises(symm.CollectiveFailure):
        eng.step()
    assert len(eng.sched.requests["a"].output_token_ids) == n_tok  # nothing from the bad step
    fake_word.value = 0
    symm.clear_host_error()


def test_async_engine_step_raises_before_emitting(fake_word):
    """Async scheduling: a step's tokens are emitted one call later, and the health check
    runs before they are - a broken step's tokens never reach a client there either."""
    from tests.test_engine import make_engine

    eng = make_engine(async_scheduling=True)
    prompt = np.random.default_rng(1).integers(3, 500, size=40).tolist()
    eng.add_request("a", prompt, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
    assert eng.step() == []               # prefill launched, its token still in flight
    outs = eng.step()                     # next step launched, the prefill's token emitted
    assert [o.request_id for o in outs] == ["a"]
    fake_word.value = 1                   # a symm kernel timed out during the step in flight
    with pytest.raises(symm.CollectiveFailure):
        eng.step()
    fake_word.value = 0
    symm.clear_host_error()


def test_check_health_is_a_no_op_without_heap(monkeypatch):
    monkeypatch.setattr(symm, "_herr_word", None)
    symm.check_health()
    assert symm.host_error() == 0


_SERVE = r"""
import ctypes, sys, time, asyncio
sys.path.insert(0, %r)
from llmd_amd.parallel import symm
from llmd_amd.serving.async_engine import AsyncEngine
from llmd_amd.engine.request import SamplingParams
from tests.test_engine import make_engine
eng = make_engine()
word = ctypes.c_uint32(1)
symm._herr_word = word
ae = AsyncEngine(eng)
async def go():
    async for o in ae.generate("r", list(range(3, 40)), SamplingParams(max_tokens=4, ignore_eos=True)):
        print("TOKEN", o.new_token_ids, flush=True)
try:
    asyncio.run(go())
except Exception as e:
    print("CLIENT_ERROR", type(e).__name__, flush=True)
time.sleep(10)
print("STILL_ALIVE", flush=True)
"""


def test_serving_loop_exits_nonzero_on_collective_failure():
    r = subprocess.run([sys.executable, "-c", _SERVE % ROOT], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 70, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "TOKEN" not in r.stdout and "STILL_ALIVE" not in r.stdout
    assert "CLIENT_ERROR CollectiveFailure" in r.stdout


@pytest.mark.gpu
def test_stalled_peer_fails_loudly_2proc():
    env = dict(os.environ, LLMD_SYMM_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0", LLMD_SYMM_TIMEOUT_S="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29651", os.path.join(ROOT, "scripts", "symm_stall_check.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["ok"] and d["raised"] and d["host_word"] == 1
    assert 1.5 <= d["kernel_s"] < 30, d
    # later collectives of the same step must not each pay the timeout
    assert d["more_s"] < 1.5, d
