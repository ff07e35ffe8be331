"""Calibration and flow-control tuning (reference
guides/recipes/router/calibration/calibration-peak-throughput.yaml,
guides/flow-control/scripts/tuning_wizard.py, guides/flow-control/tuning.md).

``calibrate``: fresh random token-ID prompts of exactly ``chunk`` tokens (so
the prefix cache always misses), ``max_tokens=1``, streamed; TTFT to first
chunk; ``PEAK_PREFILL_THROUGHPUT = chunk / median(TTFT)`` and
``TAU = R_peak * t_max``.

``recommend``: how many requests the gateway should let through to one engine.
  compute limit  N_c = floor(throughput * latency_slo)          (Little's law)
  memory limit   N_m: each request's KV footprint over its lifetime has mean
                 mu = isl' + osl/2 and variance sigma^2 = s_isl^2 + (s_osl^2/3
                 + osl^2/12) + rho*s_isl*s_osl (uniform progress through the
                 output); by the CLT the total of N requests stays below the
                 available tokens T with confidence z when
                 N*mu + z*sqrt(N)*sigma <= T -> solve the quadratic in sqrt(N).
  active batch   min(N_c, N_m);  lookahead buffer B = min(ceil(mnbt / isl),
                 ceil(0.15 * N));  gateway maxConcurrency = N + B.
"""
from __future__ import annotations

import argparse
import json
import math
import random
import statistics
import sys
import time
import urllib.error
import urllib.request
from dataclasses import asdict, dataclass
from typing import Optional


def compute_limit(throughput_rps: float, latency_s: float) -> int:
    return int(math.floor(throughput_rps * latency_s))


def memory_limit(gpu_blocks: int, block_size: int, efficiency: float = 0.9, shared_prefix: int = 0,
                 prefix_caching: bool = True, isl_mean: float = 0.0, isl_std: float = 0.0, osl_mean: float = 0.0,
                 osl_std: float = 0.0, rho: float = 0.0, z: float = 2.33) -> tuple[int, float, float]:
    """Returns (max concurrent requests, marginal isl, coefficient of variation)."""
    tokens = gpu_blocks * block_size * efficiency
    if prefix_caching and shared_prefix:
        tokens = max(0.0, tokens - shared_prefix)
        isl = max(0.0, isl_mean - shared_prefix)
    else:
        isl = isl_mean
    s_isl = isl_std if isl > 0 else 0.0
    mu = isl + osl_mean / 2.0
    var = s_isl ** 2 + osl_std ** 2 / 3.0 + osl_mean ** 2 / 12.0 + rho * s_isl * osl_std
    sigma = math.sqrt(max(0.0, var))
    if mu <= 0:
        raise ValueError("empty workload")
    # mu*x^2 + z*sigma*x - tokens = 0 with x = sqrt(N)
    disc = (z * sigma) ** 2 + 4 * mu * tokens
    x = (-z * sigma + math.sqrt(disc)) / (2 * mu)
    return int(x * x), isl, sigma / mu


def lookahead_buffer(active: int, max_num_batched_tokens: int, isl_mean: Optional[float]) -> int:
    cap = math.ceil(active * 0.15)
    if not isl_mean:
        return max(1, cap)
    return max(1, min(math.ceil(max_num_batched_tokens / max(1.0, isl_mean)), cap))


@dataclass
class Recommendation:
    compute_limit: Optional[int]
    memory_limit: Optional[int]
    bottleneck: str
    active_batch: int
    lookahead_buffer: int
    max_concurrency: int
    warnings: list


def recommend(throughput_rps: Optional[float] = None, latency_s: Optional[float] = None,
              gpu_blocks: Optional[int] = None, block_size: int = 64, max_num_batched_tokens: int = 8192,
              **mem) -> Recommendation:
    nc = compute_limit(throughput_rps, latency_s) if throughput_rps and latency_s else None
    nm, cv = None, 0.0
    if gpu_blocks:
        nm, _, cv = memory_limit(gpu_blocks, block_size, **mem)
    if nc is not None and nm is not None:
        n = min(nc, nm)
        bott = "compute (latency SLO)" if nc <= nm else "memory (KV cache)"
    elif nc is not None:
        n, bott = nc, "compute only (OOM risk)"
    elif nm is not None:
        n, bott = nm, "memory only (latency risk)"
    else:
        raise ValueError("need throughput+latency and/or KV geometry")
    if n < 1:
        raise ValueError("hardware cannot support this workload (active batch < 1)")
    b = lookahead_buffer(n, max_num_batched_tokens, mem.get("isl_mean"))
    warns = []
    if nc is not None and nc < 30:
        warns.append(f"small batch ({nc} < 30): CLT assumptions weak")
    if cv > 0.5:
        warns.append(f"heavy-tailed footprint (cv={cv:.2f} > 0.5): raise z or efficiency margin")
    return Recommendation(nc, nm, bott, n, b, n + b, warns)


# ------------------------------------------------------------- calibration
def _ttft(endpoint: str, model: str, prompt: list[int], timeout: float = 120.0) -> float:
    body = json.dumps({"model": model, "prompt": prompt, "max_tokens": 1, "stream": True,
                       "temperature": 0}).encode()
    req = urllib.request.Request(endpoint.rstrip("/") + "/v1/completions", data=body,
                                 headers={"Content-Type": "application/json"})
    t0 = time.monotonic()
    with urllib.request.urlopen(req, timeout=timeout) as r:
        for line in r:
            line = line.strip()
            if line.startswith(b"data:") and b"[DONE]" not in line:
                return time.monotonic() - t0
    raise RuntimeError("no streamed chunk received")


def calibrate(endpoint: str, model: str, chunk: int, t_max: float = 1.0, warmup: int = 5,
              measurements: int = 20, token_min: int = 100, token_max: int = 10000,
              out=sys.stdout) -> dict:
    seed = time.time_ns()  # fresh every run so a persistent KV tier never hits
    rng = random.Random(seed)
    prompt = lambda: [rng.randint(token_min, token_max) for _ in range(chunk)]  # noqa: E731
    print(f"using seed={seed} endpoint={endpoint} model={model} chunk={chunk}", file=out, flush=True)
    for i in range(warmup):
        print(f"  warmup {i + 1}: TTFT={_ttft(endpoint, model, prompt()):.4f}s", file=out, flush=True)
    samples = []
    for i in range(measurements):
        samples.append(_ttft(endpoint, model, prompt()))
        print(f"  measure {i + 1}: TTFT={samples[-1]:.4f}s", file=out, flush=True)
    med = statistics.median(samples)
    r_peak = chunk / med
    print(f"PEAK_PREFILL_THROUGHPUT={int(r_peak)}", file=out, flush=True)
    print(f"TAU={int(r_peak * t_max)}", file=out, flush=True)
    return {"median_ttft": med, "peak_prefill_throughput": r_peak, "tau": r_peak * t_max, "samples": samples}


def main(argv=None):
    p = argparse.ArgumentParser("llmd-tune")
    sub = p.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("calibrate")
    c.add_argument("--endpoint", required=True)
    c.add_argument("--model", required=True)
    c.add_argument("--chunk-size", type=int, default=8192)
    c.add_argument("--t-max", type=float, default=1.0)
    c.add_argument("--warmup", type=int, default=5)
    c.add_argument("--measurements", type=int, default=20)
    w = sub.add_parser("wizard")
    w.add_argument("--throughput", type=float, help="sustained requests/s at the SLO")
    w.add_argument("--latency", type=float, help="mean e2e latency (s) at that throughput")
    w.add_argument("--gpu-blocks", type=int)
    w.add_argument("--block-size", type=int, default=64)
    w.add_argument("--max-num-batched-tokens", type=int, default=8192)
    w.add_argument("--paged-attention-efficiency", type=float, default=0.9)
    w.add_argument("--shared-prefix", type=int, default=0)
    w.add_argument("--no-prefix-caching", action="store_true")
    w.add_argument("--isl-mean", type=float, default=0)
    w.add_argument("--isl-std", type=float, default=0)
    w.add_argument("--osl-mean", type=float, default=0)
    w.add_argument("--osl-std", type=float, default=0)
    w.add_argument("--correlation", type=float, default=0)
    w.add_argument("--z-score", type=float, default=2.33)
    a = p.parse_args(argv)
    if a.cmd == "calibrate":
        calibrate(a.endpoint, a.model, a.chunk_size, a.t_max, a.warmup, a.measurements)
        return
    mem = {}
    if a.gpu_blocks:
        mem = dict(efficiency=a.paged_attention_efficiency, shared_prefix=a.shared_prefix,
                   prefix_caching=not a.no_prefix_caching, isl_mean=a.isl_mean, isl_std=a.isl_std,
                   osl_mean=a.osl_mean, osl_std=a.osl_std, rho=a.correlation, z=a.z_score)
    r = recommend(a.throughput, a.latency, a.gpu_blocks, a.block_size, a.max_num_batched_tokens, **mem)
    print(json.dumps(asdict(r), indent=2))


if __name__ == "__main__":
    main()
