"""Two-process P/D through kvx IPC on one GPU (GPU only): the bench's pd mode
with a small model; checks the JSON result line."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pd_two_process_ipc():
    env = dict(os.environ, LLMD_BENCH_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29611", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--mode", "pd", "--prefill-gpus", "1", "--model", "small-llama",
           "--isl", "1000", "--osl", "32", "--concurrency", "8", "--steps", "16", "--warmup", "4",
           "--kv-cache-gb", "4", "--max-num-batched-tokens", "4096"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["value"] > 0 and d["config"]["parallelism"] == "pd1p1d"
    assert d["p50_ttft_s"] is not None
