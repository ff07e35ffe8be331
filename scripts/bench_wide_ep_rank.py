"""One wide-EP decode rank of DeepSeek-R1 on one GPU: a per-decode-GPU
throughput projection for the reference's wide-EP guide, which reports ~1350
output tok/s per decode GPU at ~128 concurrent requests per decode rank, ISL 2k
/ OSL 2k (/root/reference/guides/wide-ep-lws/README.md:452-465).

What runs (measured): the whole 61-layer DeepSeek-R1 decode step of ONE rank of
an EP-``ep`` deployment with DP attention:
  * MLA attention over this rank's own ``batch`` sequences at context ``ctx``
    (paged latent KV, the absorbed MLA decode kernel, hipGraphs);
  * the 3 dense layers, the shared expert and the router gate for its tokens;
  * the routed experts this rank OWNS: E/ep (+ ``redundant`` EPLB slots)
    block-fp8 experts receiving batch x top-k rows per step. Under balanced
    routing an EP rank receives exactly batch x k expert rows (its own share
    of every rank's tokens), so the preset routes this rank's tokens over its
    local experts only: the same grouped-GEMM rows, weights and bytes;
  * the fp8 LL dispatch + bf16 combine kernels of the symm heap in loopback
    (world 1): their kernel time per MoE layer.

What is modelled (not measurable on one GPU): the xGMI transfer of the
exchange. Per MoE layer a rank sends each token to ~D distinct ranks
(D = ep (1 - (1 - 1/ep)^k)), (D - D/ep) of them remote: fp8 rows + scales out,
bf16 partial rows back, spread over ep-1 point-to-point links at ``link_gbs``
each, plus ``hop_us`` of barrier latency per exchange. Reported separately so
the projection's assumption is explicit.

  python scripts/bench_wide_ep_rank.py [--ep 8] [--batch 128] [--ctx 3072] [--steps 30]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmd_amd.engine import config as C  # noqa: E402
from llmd_amd.engine.config import EngineConfig  # noqa: E402
from llmd_amd.engine.engine import LLMEngine  # noqa: E402
from llmd_amd.engine.request import SamplingParams  # noqa: E402

REF_TOK_S_PER_DECODE_GPU = 1350.0


def exchange_kernel_us(d, k, rows, E_local, iters=50):
    """fp8 dispatch + combine kernels, world-1 heap (loopback), per MoE layer."""
    from llmd_amd.parallel import symm

    heap = symm.SymmHeap(symm.SymmEP.heap_bytes(1, rows, d, k, fp8=True) + (2 << 20), 0, 1)
    sep = symm.SymmEP(heap, rows, d, k, fp8=True)
    x = torch.randn(rows, d, device="cuda").to(torch.bfloat16)
    ids = torch.stack([torch.randperm(E_local)[:k] for _ in range(rows)]).to(torch.int32).cuda()
    w = torch.rand(rows, k, device="cuda")
    y = torch.zeros(rows, d, dtype=torch.bfloat16, device="cuda")
    fn = lambda rx, rid, rw: y  # noqa: E731 - exchange only
    for _ in range(5):
        sep.moe(x, ids, w, E_local, rows, fn)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        sep.moe(x, ids, w, E_local, rows, fn)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / iters * 1e6
    err = heap.error()
    heap.close()
    return us, err


def modelled_link_us(ep, batch, d, k, link_gbs, hop_us):
    D = ep * (1 - (1 - 1 / ep) ** k)           # distinct destination ranks per token
    remote = D * (ep - 1) / ep                   # of which remote
    ng = -(-d // 128)
    out_b = batch * remote * (ng * 128 + ng * 4)  # fp8 rows + scales
    back_b = batch * remote * d * 2               # bf16 partial outputs
    links = max(ep - 1, 1)
    return (out_b + back_b) / (links * link_gbs * 1e9) * 1e6 + 2 * hop_us, D


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ep", type=int, default=8)
    ap.add_argument("--redundant", type=int, default=0, help="EPLB redundant expert slots per rank")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=3072, help="mean decode context (ISL 2k + half of OSL 2k)")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--layers", type=int, default=61)
    ap.add_argument("--kv-cache-dtype", default="auto")
    ap.add_argument("--kv-cache-gb", type=float, default=48.0)
    ap.add_argument("--link-gbs", type=float, default=50.0, help="usable one-way GB/s per xGMI link")
    ap.add_argument("--hop-us", type=float, default=8.0, help="barrier latency per exchange (us)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    base = C.get_model_config("deepseek-r1")
    E_local = base.num_local_experts // a.ep + a.redundant
    name = f"deepseek-r1-ep{a.ep}-rank"
    C._register(dataclasses.replace(base, name=name, num_local_experts=E_local, n_group=1, topk_group=1,
                                    num_hidden_layers=a.layers))
    mt = a.steps + 40 + (a.batch * a.ctx) // 8192
    cfg = EngineConfig.create(name, device="cuda", block_size=64, max_num_seqs=a.batch,
                              max_num_batched_tokens=8192, max_model_len=a.ctx + mt + 64,
                              cuda_graph_max_bs=a.batch, quantization="fp8", kv_cache_dtype=a.kv_cache_dtype,
                              kv_cache_memory_bytes=int(a.kv_cache_gb * 2**30))
    t_build = time.perf_counter()
    eng = LLMEngine(cfg)
    print(f"[ep-rank] engine built in {time.perf_counter() - t_build:.0f}s: {E_local} local experts x "
          f"{a.layers} layers, {torch.cuda.memory_allocated() / 2**30:.0f} GiB allocated", flush=True)
    rng = np.random.default_rng(0)
    sp = SamplingParams(max_tokens=mt, temperature=0.0, ignore_eos=True)
    for i in range(a.batch):
        eng.add_request(f"r{i}", rng.integers(100, 100000, size=a.ctx).tolist(), sp)
    tp = time.perf_counter()
    n = 0
    while eng.sched.num_waiting or any(not r.output_token_ids for r in eng.sched.running):
        eng.step()
        n += 1
        if n % 20 == 0:
            print(f"[ep-rank] prefill step {n} ({time.perf_counter() - tp:.0f}s)", flush=True)
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    g0 = eng.metrics.n_gen
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / a.steps * 1e3
    ran = (eng.metrics.n_gen - g0) / a.steps
    moe_layers = a.layers - base.first_k_dense_replace
    xk_us, err = exchange_kernel_us(base.hidden_size, base.num_experts_per_tok, a.batch, E_local)
    link_us, D = modelled_link_us(a.ep, a.batch, base.hidden_size, base.num_experts_per_tok, a.link_gbs,
                                  a.hop_us)
    total_ms = step_ms + moe_layers * (xk_us + link_us) / 1e3
    tok_s = ran / (total_ms / 1e3)
    res = {"model": "DeepSeek-R1 (random init, fp8 block experts, bf16 MLA)", "ep": a.ep,
           "local_experts": E_local, "batch_per_rank": a.batch, "ctx": a.ctx, "running": ran,
           "step_ms_measured": round(step_ms, 2), "exchange_kernels_us_per_layer": round(xk_us, 1),
           "exchange_link_us_per_layer_modelled": round(link_us, 1), "distinct_dest_ranks": round(D, 2),
           "moe_layers": moe_layers, "step_ms_projected": round(total_ms, 2),
           "output_tok_s_per_decode_gpu": round(tok_s, 1), "reference_tok_s_per_decode_gpu": REF_TOK_S_PER_DECODE_GPU,
           "vs_reference": round(tok_s / REF_TOK_S_PER_DECODE_GPU, 3), "symm_timeout_flag": err,
           "assumptions": f"xGMI {a.link_gbs} GB/s/link usable, {a.hop_us} us/exchange barrier, balanced routing"}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
