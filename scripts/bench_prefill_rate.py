"""Prefill-only throughput of one engine (the P/D prefill rank's job): a closed
loop of ISL-token prompts with max_tokens=1, chunked within
--max-num-batched-tokens; prints prompt tok/s and the implied output tok/s one
such rank feeds at OSL (prompt rate / ISL * OSL).
  python scripts/bench_prefill_rate.py [--model llama-3-70b] [--isl 5000] [--osl 250] [--steps 12]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmd_amd.engine.config import EngineConfig  # noqa: E402
from llmd_amd.engine.engine import LLMEngine  # noqa: E402
from llmd_amd.engine.request import SamplingParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--isl", type=int, default=5000)
    ap.add_argument("--osl", type=int, default=250)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--inflight", type=int, default=6)
    ap.add_argument("--quantization", default=None, choices=[None, "fp8", "mxfp4"])
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"])
    a = ap.parse_args()
    cfg = EngineConfig.create(a.model, device="cuda", block_size=64, max_num_seqs=64,
                              max_num_batched_tokens=a.max_num_batched_tokens, max_model_len=a.isl + 64,
                              enforce_eager=True, kv_cache_memory_bytes=40 << 30,
                              quantization=a.quantization, kv_cache_dtype=a.kv_cache_dtype)
    eng = LLMEngine(cfg)
    rng = np.random.default_rng(0)
    sp = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    n = [0]

    def add():
        n[0] += 1
        eng.add_request(f"r{n[0]}", rng.integers(100, 30000, size=a.isl).tolist(), sp)

    for _ in range(a.inflight):
        add()

    def run(k):
        for _ in range(k):
            for o in eng.step():
                if o.finished:
                    add()

    run(a.warmup)
    torch.cuda.synchronize()
    p0 = eng.metrics.n_prompt
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pt = eng.metrics.n_prompt - p0
    rate = pt / dt
    print(f"{a.model} ({a.quantization or 'bf16'}, kv {a.kv_cache_dtype}) prefill ISL {a.isl}: {pt} prompt tokens in {dt:.2f}s = {rate:.0f} tok/s "
          f"({1000 * dt / a.steps:.0f} ms/step) -> feeds {rate / a.isl * a.osl:.0f} output tok/s at OSL {a.osl}",
          flush=True)


if __name__ == "__main__":
    main()
