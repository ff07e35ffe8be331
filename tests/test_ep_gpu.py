"""Wide-EP on the GPU through the symm heap (DeepEP-LL role) with hipGraph
decode, dual-batch overlap and EPLB: scripts/ep_gpu_check.py with 2 processes
sharing cuda:0, outputs compared with a single-process engine (GPU only)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("model,flags,port", [
    ("tiny-gpt-oss", [], 29751),
    ("tiny-deepseek", ["--dbo", "--eplb"], 29752),
    # the engine path (graphs, DBO) with the chunked HT exchange and with
    # block-fp8 experts (rows quantised to e4m3 inside the dispatch kernel)
    ("tiny-deepseek", ["--backend", "symm_ht", "--dbo"], 29753),
    ("tiny-deepseek", ["--quantization", "fp8", "--dbo"], 29754),
    ("tiny-gpt-oss", ["--backend", "symm_ht", "--quantization", "fp8"], 29755)])
def test_wide_ep_symm_gpu(model, flags, port, tmp_path):
    env = dict(os.environ, LLMD_SYMM_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "scripts", "ep_gpu_check.py"),
           "--model", model, "--weights", str(tmp_path / "w.safetensors")] + flags
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=220)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    d = json.loads(lines[-1]) if lines else None
    if r.returncode != 0 or d is None or not d["ok"]:
        # torchrun's trailer hides the failing rank's traceback: keep the whole log.
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"ep_gpu_{model}.log"), "w") as f:
            f.write(r.stdout + "\n---- stderr ----\n" + r.stderr)
    assert d is not None, ("no result line (a rank raised)", r.stdout[-2000:],
                           [l for l in r.stderr.splitlines() if "rror" in l or "Traceback" in l][-20:])
    # name the failed condition: symm-heap barrier timeout vs greedy divergence
    assert all(x["timeout_flag"] == 0 for x in d["ranks"]), ("symm heap timeout flag", d["ranks"])
    assert d["ok"], ("greedy divergence beyond a near-tie", [x["diverge"] for x in d["ranks"]])
    assert r.returncode == 0, r.stderr[-4000:]
