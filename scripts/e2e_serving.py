#!/usr/bin/env python3
"""End-to-end serving measurement through the whole HTTP stack: N engine
replicas (OpenAI API servers, one process each) behind the router proxy,
driven by the load generator with a shared-prefix workload (the reference's
prefix-cache-aware routing benchmark shape, guides/optimized-baseline and
precise-prefix-cache-routing). The same load runs under several EPP
configurations so the routing policy is the only variable:

* ``prefix``  - the reference's optimized-baseline EPP config (queue 2,
  kv-util 2, prefix 3 over the approx producer, no-hit-LRU 2);
* ``precise`` - the same scorers fed by the KV-event index (engines publish
  BlockStored / BlockRemoved; precise-prefix-cache-routing);
* ``load``    - queue + kv-util scorers only (no prefix affinity);
* ``random``  - random picker.

Between configurations every engine's prefix cache is reset. Reported per
configuration: output / input tok/s, TTFT and ITL percentiles, and the
engines' prefix-cache hit rate (``vllm:prefix_cache_hits`` /
``vllm:prefix_cache_queries`` deltas). With the KV pool sized so that one
replica holds only part of the prefix groups, prefix-affine routing keeps
each group on one replica and the others thrash.

  python scripts/e2e_serving.py --model llama-3-8b --replicas 2 --device cuda
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import subprocess
import sys
import tempfile
import time
import urllib.request

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from llmd_amd.router.datalayer import parse_prometheus  # noqa: E402
from llmd_amd.tools import loadgen  # noqa: E402

CONFIGS = {
    # the reference's optimized-baseline EPP config verbatim
    # (guides/optimized-baseline/router/optimized-baseline.values.yaml): the
    # prefix-cache-scorer brings the approx producer with its defaults (autoTune)
    "prefix": """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: queue-scorer
- type: kv-cache-utilization-scorer
- type: prefix-cache-scorer
- type: no-hit-lru-scorer
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: queue-scorer
    weight: 2
  - pluginRef: kv-cache-utilization-scorer
    weight: 2
  - pluginRef: prefix-cache-scorer
    weight: 3
  - pluginRef: no-hit-lru-scorer
    weight: 2
""",
    "precise": """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: precise-prefix-cache-producer
  parameters:
    tokenProcessorConfig: {blockSize: 16}
    speculativeIndexing: true
    kvEventsConfig: {discoverPods: true}
- type: prefix-cache-scorer
- type: queue-scorer
- type: kv-cache-utilization-scorer
- type: max-score-picker
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: precise-prefix-cache-producer
  - pluginRef: prefix-cache-scorer
    weight: 3
  - pluginRef: queue-scorer
    weight: 2
  - pluginRef: kv-cache-utilization-scorer
    weight: 2
  - pluginRef: max-score-picker
""",
    "load": """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: queue-scorer
- type: kv-cache-utilization-scorer
- type: max-score-picker
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: queue-scorer
    weight: 2
  - pluginRef: kv-cache-utilization-scorer
    weight: 2
  - pluginRef: max-score-picker
""",
    "random": """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: random-picker
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: random-picker
""",
}


def _get(url, timeout=2.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.read().decode()
    except OSError:
        return None


def _post(url, body=None, timeout=30):
    req = urllib.request.Request(url, data=json.dumps(body or {}).encode(), headers={"content-type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.read()


def _wait(url, procs, timeout):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if _get(url) is not None:
            return True
        for p in procs:
            if p.poll() is not None:
                raise RuntimeError(f"process {p.args[:6]} exited with {p.returncode}")
        time.sleep(1)
    return False


def _offload_loads(ports):
    n = 0.0
    for port in ports:
        m = parse_prometheus(_get(f"http://127.0.0.1:{port}/metrics", 5) or "")
        n += sum(v for lab, v in m.get("vllm:kv_offload_blocks_total", []) if lab.get("op", "").startswith("load"))
    return n


def _prefix_counters(ports):
    hits = queries = 0.0
    for port in ports:
        m = parse_prometheus(_get(f"http://127.0.0.1:{port}/metrics", 5) or "")
        hits += sum(v for _, v in m.get("vllm:prefix_cache_hits_total", m.get("vllm:prefix_cache_hits", [])))
        queries += sum(v for _, v in m.get("vllm:prefix_cache_queries_total",
                                             m.get("vllm:prefix_cache_queries", [])))
    return hits, queries


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--replicas", type=int, default=2)
    ap.add_argument("--blocks", type=int, default=4096, help="KV blocks (16 tokens) per replica (0: sized by the engine, e.g. --kv-cache-memory-bytes)")
    ap.add_argument("--groups", type=int, default=48)
    ap.add_argument("--per-group", type=int, default=16)
    ap.add_argument("--system-len", type=int, default=2048)
    ap.add_argument("--question-len", type=int, default=128)
    ap.add_argument("--output-len", type=int, default=64)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--requests", type=int, default=768)
    ap.add_argument("--configs", default="prefix,precise,load,random")
    ap.add_argument("--kv-events-port-base", type=int, default=15556)
    ap.add_argument("--port-base", type=int, default=18200)
    ap.add_argument("--router-port", type=int, default=18100)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "e2e_serving.json"))
    ap.add_argument("--extra-engine-args", default="")
    ap.add_argument("--kv-offload-gb", type=float, default=0.0, help="host-DRAM KV tier per replica")
    ap.add_argument("--workload", default=None, help="benchmark profile (llmd_amd/tools/workloads) to run instead")
    ap.add_argument("--overrides", default="", help="benchmark profile overrides (k=v,...)")
    a = ap.parse_args()

    from llmd_amd.engine.config import get_model_config

    vocab = min(32000, get_model_config(a.model).vocab_size)
    work = tempfile.mkdtemp(prefix="llmd-e2e-")
    ports = [a.port_base + i for i in range(a.replicas)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", POD_IP="127.0.0.1")
    engines = []
    logs = []
    for i, port in enumerate(ports):
        cmd = [sys.executable, "-m", "llmd_amd.serving.api_server", "--model", a.model, "--port", str(port),
               "--device", a.device] + (["--num-gpu-blocks-override", str(a.blocks)] if a.blocks > 0 else []) + [
               "--block-size", "16",
               "--max-num-seqs", str(max(8, a.concurrency)), "--max-num-batched-tokens", "8192",
               "--max-model-len", str(a.system_len + a.question_len + a.output_len + 64),
               "--kv-events-config", json.dumps({"enable_kv_cache_events": True, "publisher": "zmq",
                                                 "endpoint": f"tcp://*:{a.kv_events_port_base + i}"})] + \
            (["--kv-offload-config", json.dumps({"cpu_bytes_to_use": int(a.kv_offload_gb * (1 << 30))})]
             if a.kv_offload_gb > 0 else []) + \
            a.extra_engine_args.split()
        log = open(os.path.join(ROOT, "gpurun_out", f"e2e_engine{i}.log"), "w")
        logs.append(log)
        engines.append(subprocess.Popen(cmd, env=dict(env, POD_PORT=str(port)), stdout=log, stderr=subprocess.STDOUT,
                                        cwd=ROOT, start_new_session=True))
    eps = {"endpoints": [{"name": f"e{i}", "address": "127.0.0.1", "port": port,
                          "labels": {"llm-d.ai/role": "prefill-decode", "llm-d.ai/model": a.model,
                                     "llm-d.ai/kv-events-port": str(a.kv_events_port_base + i)}}
                         for i, port in enumerate(ports)]}
    ep_file = os.path.join(work, "endpoints.yaml")
    with open(ep_file, "w") as f:
        yaml.safe_dump(eps, f)
    results = {"model": a.model, "replicas": a.replicas, "device": a.device, "blocks_per_replica": a.blocks,
               "kv_offload_gb": a.kv_offload_gb,
               "workload": {"groups": a.groups, "per_group": a.per_group, "system_len": a.system_len,
                            "question_len": a.question_len, "output_len": a.output_len,
                            "concurrency": a.concurrency, "requests": a.requests}, "runs": {}}
    import threading

    stop_beat = threading.Event()

    def beat():  # progress line for long runs
        t0 = time.time()
        while not stop_beat.wait(30):
            print(f"[e2e] ... {time.time() - t0:.0f}s", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    try:
        for port in ports:
            if not _wait(f"http://127.0.0.1:{port}/v1/models", engines, 600):
                raise RuntimeError(f"engine on {port} not ready")
        print(f"[e2e] {a.replicas} engines ready", flush=True)
        for run_i, name in enumerate(a.configs.split(",")):
            for port in ports:
                _post(f"http://127.0.0.1:{port}/reset_prefix_cache")
            rlog = open(os.path.join(ROOT, "gpurun_out", f"e2e_router_{name}.log"), "w")
            router = subprocess.Popen([sys.executable, "-m", "llmd_amd.router.proxy", "--port", str(a.router_port),
                                       "--endpoints-file", ep_file, "--config-text", CONFIGS[name]],
                                      env=env, stdout=rlog, stderr=subprocess.STDOUT, cwd=ROOT, start_new_session=True)
            try:
                if not _wait(f"http://127.0.0.1:{a.router_port}/health", [router], 60):
                    raise RuntimeError("router not ready")
                time.sleep(2)  # first metrics scrape of every endpoint
                h0, q0 = _prefix_counters(ports)
                l0 = _offload_loads(ports)
                cfg = {"load": {"type": "concurrent", "stages": [{"concurrency": a.concurrency,
                                                                  "num_requests": a.requests}]},
                       "api": {"type": "completion"},
                       "server": {"base_url": f"http://127.0.0.1:{a.router_port}", "model_name": a.model,
                                  "ignore_eos": True},
                       "data": {"type": "shared_prefix",
                                "shared_prefix": {"num_groups": a.groups, "num_prompts_per_group": a.per_group,
                                                  "system_prompt_len": a.system_len,
                                                  "question_len": a.question_len, "output_len": a.output_len}}}
                if a.workload:  # a shipped benchmark profile (llmd_amd.tools.benchmark) instead
                    from llmd_amd.tools import benchmark

                    _, text = benchmark.load_profile(a.workload)
                    cfg = benchmark.apply_overrides(
                        benchmark.render(text, f"http://127.0.0.1:{a.router_port}", a.model), a.overrides)
                t0 = time.time()
                rep = asyncio.run(loadgen.run(cfg, vocab=vocab, seed=1))
                wall = time.time() - t0
                if a.workload:
                    results.setdefault("stages", {})[name] = [
                        {"config": st["config"], "output_tok_s": st["throughput"]["output_tokens_per_sec"],
                         "req_s": st["throughput"]["requests_per_sec"], "failures": st["requests"]["failures"],
                         "ttft_mean_s": st["latency"]["time_to_first_token"]["mean"],
                         "ttft_p90_s": st["latency"]["time_to_first_token"]["p90"],
                         "itl_mean_s": st["latency"]["inter_token_latency"]["mean"]} for st in rep["stages"]]
                    for st in results["stages"][name]:
                        print(f"[e2e] {name} stage " + json.dumps(st), flush=True)
                h1, q1 = _prefix_counters(ports)
                l1 = _offload_loads(ports)
                s = rep["summary"]
                out = {"wall_s": wall, "requests": s["requests"]["total"], "failures": s["requests"]["failures"],
                       "output_tok_s": s["throughput"]["output_tokens_per_sec"],
                       "input_tok_s": s["throughput"]["input_tokens_per_sec"],
                       "ttft_p50_s": s["latency"]["time_to_first_token"]["p50"],
                       "ttft_p90_s": s["latency"]["time_to_first_token"]["p90"],
                       "itl_p50_s": s["latency"]["inter_token_latency"]["p50"],
                       "prefix_hit_rate": (h1 - h0) / (q1 - q0) if q1 > q0 else None,
                       "offload_blocks_loaded": l1 - l0}
                results["runs"][name if name not in results["runs"] else f"{name}#{run_i}"] = out
                print(f"[e2e] {name}: " + json.dumps(out), flush=True)
            finally:
                os.killpg(router.pid, signal.SIGTERM)
                router.wait(30)
                rlog.close()
    finally:
        stop_beat.set()
        for p in engines:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        for p in engines:
            try:
                p.wait(60)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        for f in logs:
            f.close()
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)
    print(json.dumps(results), flush=True)


if __name__ == "__main__":
    main()
