#!/usr/bin/env python3
"""Serving benchmark: Llama-3-70B, ISL 5000 / OSL 250 (the reference's P/D
benchmark shape, guides/pd-disaggregation/README.md:336-520), bf16, random-init
weights, synthetic random-token prompts.

A *step* is one engine iteration on every rank (continuous batching: decode
tokens of all running requests + chunked-prefill tokens of new ones, within
``--max-num-batched-tokens``). Each rank keeps ``--concurrency`` requests in
flight (closed loop: a finished request is immediately replaced), W warmup
steps bring the batch to steady state, then exactly K steps are timed between
barrier+synchronize brackets; the slowest rank's time is used.

Modes (default ``auto``: agg for N < 8, pd for N >= 8)
  agg : every GPU is an independent aggregated replica (dp N) - the
        optimized-baseline topology; per-GPU work fixed as N grows (weak scaling).
  pd  : ranks [0, P) prefill, [P, N) decode (P = 3N/4 unless --prefill-gpus),
        decode ranks paired into TP2 replicas when they can (--decode-tp);
        KV moves over xGMI (kvx VMM-chunked IPC pool). Measured on one
        MI355X: a 70B bf16 prefill rank feeds 481-497 output tok/s
        (scripts/bench_prefill_rate.py), a TP1 decode replica at batch 64
        sustains 1349 tok/s (47.5 ms/step) and one aggregated GPU 358 tok/s.
        So 1P1D (N=2) idles the decoder and 3P1D (N=4) is decode-bound at
        ~1350 < 4 x 358: both run aggregated. From N=8, 6P + one TP2 decode
        replica (two GPUs, batch 128 in ~40 ms + the TP all-reduces) balances
        the six prefill GPUs at ~2900-3000 tok/s, above 8 aggregated GPUs
        (~2860), with the prefill of every request on a dedicated GPU. The
        reference tunes the P:D ratio per workload the same way
        (guides/pd-disaggregation/README.md:15-33).

Multi-GPU robustness (N > 1): every process group has an explicit timeout
(LLMD_DIST_TIMEOUT, default 1800 s) and, before any engine starts, a
pre-flight (llmd_amd/parallel/preflight.py) proves peer access, IPC and VMM
pulls, the symm all-reduce (vs RCCL, bit for bit) and the symm EP exchange (vs
the RCCL all_to_all path) on this node; a failure exits non-zero with the
failing check and ranks. Under the bench the kvx connector may not degrade a
P/D pull to TCP (require_ipc): a failed IPC path is an error, never a silent
1.6 GB msgpack per request.

At N = 8 the P/D run is followed by BASELINE.json's literal split, 2P + 6D
(``alt_split`` in the JSON; --alt-split none disables), and every result
carries ``output_tok_s_per_gpu`` (whole job / N) next to the per-decode-GPU
figure.

Output: one JSON line on rank 0 (see README "bench.py contract").
"""
from __future__ import annotations

import argparse
import collections
import datetime
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from llmd_amd.tools import steady

METRIC = "output tok/s per decode GPU + p50 TTFT, Llama-3-70B P/D-disagg on 8×MI355X"
REF_CONTEXT = ("reference publishes no Llama-3-70B number; its P/D headline is gpt-oss-120b on 16xH200 "
               "(8 P TP1 + 2 D TP4): 12236.6 output tok/s total = 1529.6 per decode GPU, p50 TTFT 1.264 s "
               "(guides/pd-disaggregation/README.md:336-460)")


# The reference's published P/D run (guides/pd-disaggregation/README.md:336-460):
# gpt-oss-120b, ISL ~5150 / OSL ~250, 16 H200 = 8 prefill TP1 + 2 decode TP4.
REF_GPTOSS_TOK_S, REF_GPTOSS_GPUS = 12236.6, 16


def _metric(model: str) -> str:
    if model == "llama-3-70b":
        return METRIC
    return f"output tok/s per decode GPU + p50 TTFT, {model}"


def _reference(model: str, value: float, n_gpus: int) -> dict:
    if model != "gpt-oss-120b":
        return {"reference_context": REF_CONTEXT}
    per_gpu = REF_GPTOSS_TOK_S / REF_GPTOSS_GPUS
    return {"reference_context": "reference gpt-oss-120b P/D on 16xH200 (mxfp4 weights): 12236.6 output tok/s "
                                 "= 764.8 per GPU (guides/pd-disaggregation/README.md:336-460)",
            "reference_output_tok_s_per_gpu": round(per_gpu, 1),
            "output_tok_s_per_gpu_vs_reference": round(value / n_gpus / per_gpu, 3)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--model", default="llama-3-70b")
    p.add_argument("--isl", type=int, default=5000)
    p.add_argument("--osl", type=int, default=250)
    p.add_argument("--concurrency", type=int, default=64, help="requests in flight per GPU")
    p.add_argument("--max-num-batched-tokens", type=int, default=8192)
    p.add_argument("--block-size", type=int, default=64)
    p.add_argument("--mode", default="auto", choices=["auto", "agg", "pd"],
                   help="auto: aggregated replicas on N < 8, P/D disaggregation (3/4 prefill ranks) on N >= 8")
    p.add_argument("--prefill-gpus", type=int, default=0, help="pd mode: number of prefill ranks")
    p.add_argument("--decode-tp", type=int, default=0,
                   help="pd mode: TP degree of each decode replica (0 = 2 when the decode ranks pair up, else 1)")
    p.add_argument("--enforce-eager", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--gpu-memory-utilization", type=float, default=0.92)
    p.add_argument("--kv-cache-gb", type=float, default=None)
    p.add_argument("--json-out", default=None)
    p.add_argument("--quantization", default=None, choices=[None, "fp8", "mxfp4"],
                   help="fp8 = W8A8 linears (the reference AMD recipe serves Llama-3.3-70B-FP8); default bf16")
    p.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"])
    p.add_argument("--no-async-scheduling", action="store_true",
                   help="step synchronously (default: step N+1 launched before step N's tokens reach the host)")
    p.add_argument("--alt-split", default="auto",
                   help="pd mode at N=8: also run this P:D split after the main one ('2p6d', BASELINE.json's "
                        "literal config; 'auto' = 2p6d when N=8 and the main split differs; 'none' = skip)")
    p.add_argument("--no-preflight", action="store_true", help="skip the N>1 cross-GPU pre-flight checks")
    p.add_argument("--pd-route", default="router", choices=["router", "direct"],
                   help="pd mode: requests go client -> router (EPP, the reference's P/D config) -> decode "
                        "routing sidecar -> prefill + kvx pull (router), or through an in-process sidecar loop "
                        "on each decode driver (direct)")
    p.add_argument("--pd-decider", default="always", choices=["always", "load-aware"],
                   help="pd mode, routed: the EPP's P/D decider (always-disagg = the reference config)")
    p.add_argument("--open-loop-rate", type=float, default=0.0,
                   help="pd mode, routed: Poisson request rate of the open-loop phase (0 = 0.9 x closed-loop rate)")
    p.add_argument("--open-loop-requests", type=int, default=0)
    p.add_argument("--fp8-extra", default="auto", choices=["auto", "off"],
                   help="agg mode, 1 GPU, bf16 run: also measure the reference AMD recipe's precision (W8A8 fp8 "
                        "linears + fp8 KV) in a child process and report it under 'fp8' (the bf16 figure stays "
                        "the value)")
    return p.parse_args()


def dist_timeout() -> datetime.timedelta:
    return datetime.timedelta(seconds=int(os.environ.get("LLMD_DIST_TIMEOUT", "1800")))


def _sync(a):
    if a.device == "cuda":
        torch.cuda.synchronize()


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    a = parse()
    if os.environ.get("LLMD_BENCH_STACKS"):
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["LLMD_BENCH_STACKS"]), repeat=True)
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != a.gpus and world > 1:
        log(rank, f"warning: WORLD_SIZE={world} != --gpus {a.gpus}")
    # LLMD_BENCH_DEVICE pins every rank to one GPU (multi-process rehearsal on a
    # 1-GPU box); RCCL refuses duplicate GPUs, so that mode uses gloo for control.
    forced = os.environ.get("LLMD_BENCH_DEVICE")
    a.device = "cpu" if forced == "cpu" else "cuda"  # cpu: logic rehearsal with tiny models
    dev = local_rank if forced in (None, "cpu") else int(forced)
    if a.device == "cuda":
        torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if forced is None:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev),
                                    timeout=dist_timeout())
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=dist_timeout())
        if a.device == "cuda" and not a.no_preflight:
            from llmd_amd.parallel import preflight

            # all ranks on one GPU (rehearsal): no peers, no RCCL - the IPC / VMM / symm paths only
            checks = preflight.CHECKS if forced is None else ("ipc", "vmm")
            try:
                preflight.run(rank, world, torch.device("cuda", dev), checks=checks,
                              cpu_group=dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=300)),
                              log=lambda m: print(m, file=sys.stderr, flush=True))
            except preflight.PreflightError as e:
                print(f"[bench rank {rank}] PRE-FLIGHT FAILED: {e}", file=sys.stderr, flush=True)
                sys.exit(3)

    if a.mode == "auto":
        a.mode = "pd" if world >= 8 else "agg"
    if a.mode == "pd":
        from llmd_amd.bench_pd import run_pd

        res = run_pd(a, rank, world, local_rank, log)
        alt = _alt_split(a, rank, world, local_rank, log, res)
        if rank == 0 and res is not None:
            value = res["gen"] / res["elapsed"]
            out = {
                "metric": _metric(a.model), "value": round(value, 2), "unit": "output tok/s (whole job)",
                "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": round(1000 * res["elapsed"] / a.steps, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None,
                "dtype": {"fp8": "fp8", "mxfp4": "mxfp4 experts + fp8"}.get(a.quantization, "bf16"),
                "data": "synthetic (random token prompts, random-init weights)",
                "config": {"model": "Llama-3-70B" if a.model == "llama-3-70b" else a.model,
                           "global_batch": a.concurrency * res["decode_ranks"], "seq_len": a.isl,
                           "isl": a.isl, "osl": a.osl,
                           "parallelism": f"pd{res['prefill_ranks']}p{res['decode_ranks']}d"
                                          + (f"-dtp{res['decode_tp']}" if res.get("decode_tp", 1) > 1 else ""),
                           "max_num_batched_tokens": a.max_num_batched_tokens, "block_size": a.block_size,
                           "kv_transfer": "kvx ipc over xGMI"},
                "output_tok_s_per_decode_gpu": round(value / res["decode_ranks"], 2),
                "output_tok_s_per_gpu": round(value / world, 2),
                "p50_ttft_s": round(res["p50_ttft"], 4) if res["p50_ttft"] is not None else None,
                "kv_transfer_failures": res.get("kv_failures", 0),
                **{k: res[k] for k in ("route", "open_loop", "router_pd_decisions", "sidecar_pd_requests",
                                       "sidecar_fallbacks", "steady_state", "ttft_source") if k in res},
                **_reference(a.model, value, world),
            }
            if "ttft_p90" in res:
                out["p90_ttft_s"] = round(res["ttft_p90"], 4)
            if alt is not None:
                out["alt_split"] = alt
            line = json.dumps(out)
            print(line, flush=True)
            if a.json_out:
                with open(a.json_out, "w") as f:
                    f.write(line + "\n")
        dist.barrier()
        dist.destroy_process_group()
        return

    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    # prompt + up to 2 x OSL: the steady-state re-stagger (tools/steady.py) gives
    # a request that already generated g tokens during setup up to OSL more
    max_len = a.isl + 2 * a.osl + 64
    cfg = EngineConfig.create(
        a.model, device=a.device, block_size=a.block_size, max_num_seqs=a.concurrency,
        max_num_batched_tokens=a.max_num_batched_tokens, max_model_len=max_len,
        enforce_eager=a.enforce_eager, seed=a.seed + rank, enable_prefix_caching=True,
        cuda_graph_max_bs=a.concurrency, gpu_memory_utilization=a.gpu_memory_utilization,
        kv_cache_memory_bytes=int(a.kv_cache_gb * 2**30) if a.kv_cache_gb else None,
        quantization=a.quantization, kv_cache_dtype=a.kv_cache_dtype,
        async_scheduling=not a.no_async_scheduling)
    t0 = time.time()
    eng = LLMEngine(cfg)
    eng_async = eng.async_sched
    _sync(a)
    log(rank, f"engine up in {time.time() - t0:.1f}s: {cfg.model_config.name}, "
              f"{eng.runner.num_blocks} KV blocks x {a.block_size}")
    vocab = cfg.model_config.vocab_size
    rng = np.random.default_rng(1234 + rank)
    nreq = [0]

    def new_request(max_tokens):
        toks = rng.integers(100, vocab - 100, size=a.isl).tolist()
        nreq[0] += 1
        eng.add_request(f"r{rank}-{nreq[0]}", toks,
                        SamplingParams(max_tokens=max_tokens, temperature=0.0, ignore_eos=True))

    # Setup (untimed, not part of warmup): admit C requests with staggered output
    # lengths, replacing each finished one at once (closed loop, as in the timed
    # region), and run until nothing waits and every running request is past its
    # prefill. Completions are then spread evenly over the next OSL steps, so
    # warmup/timed steps see steady-state serving (decodes + one new prefill per
    # OSL/C steps) instead of the initial all-prefill ramp or a refill burst.
    for i in range(a.concurrency):
        new_request(max(1, int(a.osl * (i + 1) / a.concurrency)))
    ts = time.time()
    setup_steps = 0
    t_note = ts
    # With C > OSL about one request completes per step, so a replacement always
    # waits at the check: then only this step's replacements may still wait.
    may_wait = a.concurrency > a.osl
    while setup_steps < 100000:
        added = 0
        for o in eng.step():
            if o.finished:
                new_request(a.osl)
                added += 1
        setup_steps += 1
        if time.time() - t_note > 30:  # progress for long setups (silent runs read as hung)
            t_note = time.time()
            log(rank, f"setup: {setup_steps} steps, {len(eng.sched.running)} running, "
                      f"{eng.sched.num_waiting} waiting")
        if eng.sched.num_waiting <= (added if may_wait else 0) and \
                all(r.output_token_ids for r in eng.sched.running):
            break
    # Steady-state phase: the admission ramp bunches the remaining output
    # lengths, so completions (and the replacement prefills) would arrive late
    # and the window would under-sample prefill steps. Re-space them to exactly
    # C/OSL per step (tools/steady.py).
    longest = steady.restagger(eng.sched.running, a.osl, a.concurrency)
    assert a.isl + longest <= max_len, (longest, max_len)
    _sync(a)
    log(rank, f"setup: {setup_steps} steps in {time.time() - ts:.1f}s (batch filled to {a.concurrency}, "
              f"completions re-spaced to {a.concurrency}/{a.osl} per step)")

    step_tokens = []
    step_ms = collections.defaultdict(list)  # step size -> wall ms (a step ends in a host sync on sampling)

    prev_n = [0]

    def run_steps(n):
        for _ in range(n):
            ts0 = time.perf_counter()
            for o in eng.step():
                if o.finished:
                    new_request(a.osl)
            # async scheduling: a call returns once the PREVIOUS step finished on the device
            # (the one it launched is still running), so its wall time is that step's
            k = prev_n[0] if eng_async else eng.last_num_tokens
            prev_n[0] = eng.last_num_tokens
            step_tokens.append(eng.last_num_tokens)
            step_ms[k].append(1000 * (time.perf_counter() - ts0))

    # warmup
    tw = time.time()
    run_steps(a.warmup)
    _sync(a)
    log(rank, f"warmup {a.warmup} steps in {time.time() - tw:.1f}s")
    # timed
    eng.metrics.ttfts.clear()
    gen0 = eng.metrics.n_gen
    prompt0 = eng.metrics.n_prompt
    if world > 1:
        dist.barrier()
    _sync(a)
    t1 = time.perf_counter()
    step_tokens.clear()
    step_ms.clear()
    run_steps(a.steps)
    _sync(a)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t1
    hist = collections.Counter(step_tokens)
    log(rank, "timed step sizes (tokens: steps, mean ms): " + ", ".join(
        f"{k}: {v} x {statistics.mean(step_ms[k]) if step_ms.get(k) else float('nan'):.1f}"
        for k, v in sorted(hist.items())))
    gen = eng.metrics.n_gen - gen0
    ptoks = eng.metrics.n_prompt - prompt0
    ttfts = list(eng.metrics.ttfts)
    stats = torch.tensor([elapsed, gen, ptoks, len(ttfts)], dtype=torch.float64,
                         device="cuda" if forced is None else "cpu")
    all_ttft = ttfts
    n_prefills = len(ttfts)  # requests whose first token (prefill end) fell in the window
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        gen, ptoks = float(sm[1]), float(sm[2])
        n_prefills = int(sm[3])
        gathered = [None] * world
        dist.all_gather_object(gathered, ttfts)
        all_ttft = [t for g in gathered for t in g]
    value = gen / elapsed
    p50 = statistics.median(all_ttft) if all_ttft else None
    n_decode_gpus = world if a.mode == "agg" else world - a.prefill_gpus
    result = {
        "metric": _metric(a.model),
        "value": round(value, 2),
        "unit": "output tok/s (whole job)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000 * elapsed / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"fp8": "fp8", "mxfp4": "mxfp4 experts + fp8"}.get(a.quantization, "bf16"),
        "data": "synthetic (random token prompts, random-init weights)",
        "config": {"model": "Llama-3-70B" if a.model == "llama-3-70b" else a.model,
                   "global_batch": a.concurrency * world, "seq_len": a.isl, "isl": a.isl, "osl": a.osl,
                   "parallelism": f"dp{world}" if a.mode == "agg" else f"pd{a.prefill_gpus}p{world - a.prefill_gpus}d",
                   "max_num_batched_tokens": a.max_num_batched_tokens, "block_size": a.block_size,
                   "graphs": not a.enforce_eager, "kv_cache_dtype": a.kv_cache_dtype,
                   "async_scheduling": eng_async},
        "output_tok_s_per_decode_gpu": round(value / max(1, n_decode_gpus), 2),
        "output_tok_s_per_gpu": round(value / world, 2),
        "p50_ttft_s": round(p50, 4) if p50 is not None else None,
        "prefill_tok_s": round(ptoks / elapsed, 1),
        # conservation check: a steady-state window of K steps holds K*C/OSL prefills per replica
        "steady_state": steady.window_report(n_prefills, a.steps * world, a.concurrency, a.osl),
        **_reference(a.model, value, world),
    }
    if rank == 0 and world == 1 and a.device == "cuda" and a.quantization is None and a.fp8_extra == "auto":
        del eng
        import gc

        gc.collect()
        torch.cuda.empty_cache()
        log(rank, f"bf16 engine released: {torch.cuda.memory_reserved() / 2**30:.1f} GiB still reserved")
        result["fp8"] = _fp8_extra(a)
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _fp8_extra(a) -> dict:
    """The same bench at the reference AMD P/D recipe's precision (amd/Llama-3.3-70B-Instruct-FP8-KV:
    W8A8 fp8 linears, fp8 KV cache; guides/pd-disaggregation/modelserver/amd/vllm/base/patch-decode.yaml:13),
    run as a CHILD process (clean GPU memory; a failure or timeout is reported, never loses the bf16
    result). Same steps / warmup / shapes."""
    import subprocess
    import tempfile

    with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as tf:
        out = tf.name
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", str(a.steps), "--warmup",
           str(a.warmup), "--model", a.model, "--isl", str(a.isl), "--osl", str(a.osl), "--concurrency",
           str(a.concurrency), "--max-num-batched-tokens", str(a.max_num_batched_tokens), "--block-size",
           str(a.block_size), "--quantization", "fp8", "--kv-cache-dtype", "fp8", "--fp8-extra", "off",
           "--json-out", out] + (["--enforce-eager"] if a.enforce_eager else [])
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    t0 = time.time()
    try:
        r = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                           timeout=float(os.environ.get("LLMD_BENCH_FP8_TIMEOUT", "420")))
        if r.returncode != 0:
            return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-400:]}
        with open(out) as f:
            d = json.loads(f.read())
    except (subprocess.TimeoutExpired, OSError, ValueError) as e:
        return {"error": repr(e)[:300]}
    finally:
        try:
            os.unlink(out)
        except OSError:
            pass
    log(0, f"fp8 extra: {d['value']} tok/s in {time.time() - t0:.0f}s")
    return {"value": d["value"], "ms_per_step": d["ms_per_step"], "p50_ttft_s": d["p50_ttft_s"],
            "prefill_tok_s": d["prefill_tok_s"], "steady_state": d["steady_state"], "dtype": "fp8",
            "kv_cache_dtype": "fp8", "quantization": "W8A8 fp8 linears (per-token x per-channel), fp8 KV",
            **({k: d[k] for k in ("output_tok_s_per_gpu_vs_reference",) if k in d})}


def _alt_split(a, rank, world, local_rank, log, main_res):
    """BASELINE.json's literal P/D split (2P + 6D at N = 8) after the main run, same
    steps; failures are reported in the JSON, never lost with the main result."""
    want = a.alt_split
    if want == "auto":
        want = "2p6d" if world == 8 else "none"
    if want in ("none", ""):
        return None
    try:
        p_n = int(want.split("p")[0])
        d_n = int(want.split("p")[1].rstrip("d"))
    except (ValueError, IndexError):
        return {"error": f"bad --alt-split {want!r}"} if rank == 0 else None
    if p_n + d_n != world or p_n == (a.prefill_gpus or (3 * world) // 4):
        return None
    import gc

    from llmd_amd.bench_pd import run_pd

    gc.collect()
    if a.device == "cuda":
        torch.cuda.empty_cache()
    b = argparse.Namespace(**vars(a))
    b.prefill_gpus, b.decode_tp = p_n, 0
    # few prefill GPUs: the load-aware decider lets decoders prefill locally while every
    # prefill queue is deep (router/plugins/scheduling.py LoadAwarePDDecider)
    b.pd_decider = os.environ.get("LLMD_ALT_PD_DECIDER", "load-aware")
    os.environ["LLMD_PD_BASE_PORT"] = str(int(os.environ.get("LLMD_PD_BASE_PORT", "18200")) + 100)
    try:
        r = run_pd(b, rank, world, local_rank, log)
    except Exception as e:  # noqa: BLE001 - the main result must survive
        print(f"[bench rank {rank}] alt split {want} failed: {e!r}", file=sys.stderr, flush=True)
        return {"split": want, "error": repr(e)} if rank == 0 else None
    if rank != 0 or r is None:
        return None
    v = r["gen"] / r["elapsed"]
    return {"split": want, "parallelism": f"pd{r['prefill_ranks']}p{r['decode_ranks']}d"
                                          + (f"-dtp{r['decode_tp']}" if r.get("decode_tp", 1) > 1 else ""),
            "value": round(v, 2), "output_tok_s_per_decode_gpu": round(v / r["decode_ranks"], 2),
            "output_tok_s_per_gpu": round(v / world, 2), "ms_per_step": round(1000 * r["elapsed"] / a.steps, 3),
            "p50_ttft_s": round(r["p50_ttft"], 4) if r["p50_ttft"] is not None else None,
            "pd_decider": b.pd_decider,
            **{k: r[k] for k in ("open_loop", "router_pd_decisions", "sidecar_pd_requests") if k in r}}


if __name__ == "__main__":
    main()
