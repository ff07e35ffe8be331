"""Decode-only step time of one engine (the P/D decode rank's job): B
sequences at context ~ISL decode with hipGraphs; prints ms/step and tok/s.
  python scripts/bench_decode.py [--model llama-3-70b] [--batch 64] [--isl 5000] [--steps 50]"""
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
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--isl", type=int, default=5000)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--kv-cache-dtype", default="auto")
    ap.add_argument("--host-profile", action="store_true", help="cProfile 20 steps (host-side cost ranking)")
    ap.add_argument("--tp-shard", type=int, default=1,
                    help="emulate one rank of a TP-N replica on one GPU: heads, FFN and vocab divided by N "
                         "(the rank's GEMM/attention/KV work; the TP all-reduces are not included)")
    ap.add_argument("--kv-cache-gb", type=float, default=None)
    ap.add_argument("--no-async-scheduling", action="store_true")
    a = ap.parse_args()
    if a.tp_shard > 1:
        import dataclasses

        from llmd_amd.engine import config as C

        mc = C.get_model_config(a.model)
        n = a.tp_shard
        C._register(dataclasses.replace(
            mc, name=f"{a.model}-tp{n}-shard", head_dim=mc.head_dim, num_attention_heads=mc.num_attention_heads // n,
            num_key_value_heads=mc.num_key_value_heads // n, intermediate_size=mc.intermediate_size // n,
            vocab_size=mc.vocab_size // n))
        a.model = f"{a.model}-tp{n}-shard"
    # requests admitted early decode during the whole chunked-prefill phase
    # (~batch*isl/8192 steps): size max_tokens so none finishes before the end
    # of the timed window (the batch must stay full while it is timed)
    mt = a.steps + 40 + (a.batch * a.isl) // 8192
    cfg = EngineConfig.create(a.model, device="cuda", block_size=64, max_num_seqs=a.batch,
                              max_num_batched_tokens=8192, max_model_len=a.isl + mt + 64,
                              cuda_graph_max_bs=a.batch, quantization=a.quantization,
                              kv_cache_dtype=a.kv_cache_dtype, async_scheduling=not a.no_async_scheduling,
                              kv_cache_memory_bytes=int(a.kv_cache_gb * 2**30) if a.kv_cache_gb else None)
    eng = LLMEngine(cfg)
    tstart = time.perf_counter()
    rng = np.random.default_rng(0)
    sp = SamplingParams(max_tokens=mt, temperature=0.0, ignore_eos=True)
    for i in range(a.batch):
        eng.add_request(f"r{i}", rng.integers(100, 30000, size=a.isl).tolist(), sp)
    while eng.sched.num_waiting or any(not r.output_token_ids for r in eng.sched.running):
        eng.step()
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g0 = eng.metrics.n_gen
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    ran = (eng.metrics.n_gen - g0) / a.steps
    if ran < a.batch:
        print(f"WARNING: only {ran:.1f} of {a.batch} sequences decoded per timed step", flush=True)
    if a.host_profile:
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        for _ in range(20):
            eng.step()
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    print(f"{a.model} q={a.quantization} kv={a.kv_cache_dtype} async={not a.no_async_scheduling} decode batch={a.batch} ctx~{a.isl}: "
          f"{dt * 1e3:.2f} ms/step  {ran / dt:.0f} tok/s (running {ran:.0f}) (prefill phase {t0 - tstart:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
