"""bench.py contract on CPU (LLMD_BENCH_DEVICE=cpu, tiny model): one JSON line
with the driver's keys, exactly K timed steps, and a setup phase that ends
when more requests are in flight than output tokens (about one completion per
step, so a replacement always waits at the setup check)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = dict(os.environ, LLMD_BENCH_DEVICE="cpu")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "tiny-llama", "--enforce-eager",
                        "--block-size", "16", "--max-num-batched-tokens", "512", *args],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


def test_bench_json_line_contract():
    d, err = _bench("--isl", "48", "--osl", "8", "--concurrency", "4", "--steps", "6", "--warmup", "2")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["steps"] == 6 and d["warmup"] == 2 and d["n_gpus"] == 1 and d["value"] > 0
    assert d["config"]["parallelism"] == "dp1" and d["dtype"] == "bf16"
    assert "timed step sizes" in err


def test_bench_setup_ends_with_more_in_flight_than_output_tokens():
    d, err = _bench("--isl", "16", "--osl", "4", "--concurrency", "24", "--steps", "4", "--warmup", "1")
    assert "batch filled to 24" in err and d["value"] > 0
