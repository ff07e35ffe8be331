"""Benchmark CLI (the ``llmdbenchmark run`` flow of
helpers/benchmark.md:26-201 for an already-deployed stack).

  python -m llmd_amd.tools.benchmark [--workspace DIR] [--spec guides/<name>] run \\
      --endpoint-url URL --model MODEL --workload shared_prefix_synthetic.yaml \\
      [--harness inference-perf] [--overrides k=v,...] [--analyze]
  python -m llmd_amd.tools.benchmark list-workloads

Workload profiles are inference-perf YAML (``llmd_amd/tools/workloads/``, or a
path) with the ``REPLACE_ENV_LLMDBENCH_*`` tokens of the reference's profiles;
``--overrides`` sets dotted keys (``load.stages.0.rate=5``,
``data.shared_prefix.num_groups=64``). The driver is the repo's load
generator (streamed OpenAI completions, token-id prompts of exact length).

Workspace layout (helpers/benchmark.md "Workspace and results layout")::

  <workspace>/runner-<ts>/plan/<profile>.yaml            rendered profile
  <workspace>/runner-<ts>/results/<experiment-id>/
      stage_<n>_lifecycle_metrics.json, summary_lifecycle_metrics.json,
      per_request_lifecycle_metrics.json, benchmark_report,_stage_<n>.yaml,
      config.yaml, <profile>.yaml, stdout.log, analysis/ (--analyze)

``benchmark_report`` follows the cross-harness schema shape (scenario, load,
metrics: requests / latency / throughput with units).
"""
from __future__ import annotations

import argparse
import asyncio
import copy
import json
import os
import sys
import time
from typing import Optional

import yaml

from . import loadgen

WORKLOADS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "workloads")
HARNESSES = ("inference-perf", "guidellm", "vllm-benchmark", "inferencemax")


def list_workloads() -> list[str]:
    return sorted(f for f in os.listdir(WORKLOADS) if f.endswith(".yaml"))


def load_profile(name: str) -> tuple[str, str]:
    """(profile name, text): a path, or a shipped profile (``.yaml`` / ``.yaml.in``)."""
    if os.path.exists(name):
        with open(name) as f:
            return os.path.basename(name), f.read()
    for cand in (name, name + ".in", name[:-3] if name.endswith(".in") else None):
        if cand and os.path.exists(os.path.join(WORKLOADS, cand)):
            with open(os.path.join(WORKLOADS, cand)) as f:
                return cand, f.read()
    raise FileNotFoundError(f"workload {name!r} not found; shipped: {', '.join(list_workloads())}")


def render(text: str, endpoint: str, model: str) -> dict:
    text = text.replace("REPLACE_ENV_LLMDBENCH_HARNESS_STACK_ENDPOINT_URL", endpoint.rstrip("/"))
    text = text.replace("REPLACE_ENV_LLMDBENCH_DEPLOY_CURRENT_MODEL", model)
    return yaml.safe_load(text)


def _coerce(v: str):
    try:
        return yaml.safe_load(v)
    except yaml.YAMLError:
        return v


def _split_top(s: str) -> list[str]:
    """Split on commas outside brackets / braces (values may be YAML flow lists)."""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "[{":
            depth += 1
        elif ch in "]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur))
    return [x.strip() for x in out if x.strip()]


def apply_overrides(cfg: dict, overrides: str) -> dict:
    cfg = copy.deepcopy(cfg)
    for kv in _split_top(overrides or ""):
        if "=" not in kv:
            raise ValueError(f"override {kv!r} is not key=value")
        k, v = kv.split("=", 1)
        parts = k.split(".")
        cur = cfg
        for i, p in enumerate(parts[:-1]):
            nxt = parts[i + 1]
            if isinstance(cur, list):
                cur = cur[int(p)]
            else:
                if p not in cur:
                    cur[p] = [] if nxt.isdigit() else {}
                cur = cur[p]
        last = parts[-1]
        if isinstance(cur, list):
            cur[int(last)] = _coerce(v)
        else:
            cur[last] = _coerce(v)
    return cfg


def _lat(stats: dict) -> dict:
    return {k: stats.get(k) for k in ("mean", "p50", "p90", "p95", "p99", "min", "max")} | \
        {"units": stats.get("units", "s")}


def benchmark_report(summary: dict, cfg: dict, stage: Optional[int], model: str, harness: str) -> dict:
    """The harness-agnostic report for one stage (or the whole run)."""
    load = cfg.get("load", {})
    st_cfg = (load.get("stages") or [{}])[stage] if stage is not None else None
    lat = summary["latency"]
    return {
        "version": "0.1",
        "scenario": {"model": {"name": model}, "load": {"harness": harness, "type": load.get("type"),
                                                        "stage": stage, "config": st_cfg,
                                                        "data": cfg.get("data", {})},
                     "host": {"accelerator": os.environ.get("LLMD_ACCELERATOR", "MI355X")}},
        "metrics": {
            "time": {"duration": summary.get("duration_s"), "units": "s"},
            "requests": {"total": summary["requests"]["total"], "failures": summary["requests"]["failures"],
                         "input_length": summary["requests"]["input_length"],
                         "output_length": summary["requests"]["output_length"]},
            "latency": {"time_to_first_token": _lat(lat["time_to_first_token"]),
                        "inter_token_latency": _lat(lat["inter_token_latency"]),
                        "time_per_output_token": _lat(lat["time_per_output_token"]),
                        "request_latency": _lat(lat["request_latency"])},
            "throughput": {"requests_per_sec": summary["throughput"]["requests_per_sec"],
                           "input_tokens_per_sec": summary["throughput"]["input_tokens_per_sec"],
                           "output_tokens_per_sec": summary["throughput"]["output_tokens_per_sec"],
                           "total_tokens_per_sec": summary["throughput"]["total_tokens_per_sec"]},
        },
    }


def analyze(per_req: list[dict], out_dir: str) -> list[str]:
    """Per-request distribution plots (TTFT, ITL, e2e, output length)."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    os.makedirs(out_dir, exist_ok=True)
    ok = [r for r in per_req if r["ok"]]
    series = {"ttft": [r["time_to_first_token"] for r in ok],
              "request_latency": [r["request_latency"] for r in ok],
              "output_tokens": [r["output_tokens"] for r in ok],
              "itl_all_tokens": [x for r in ok for x in r["inter_token_latencies"]]}
    files = []
    for name, xs in series.items():
        if not xs:
            continue
        fig, ax = plt.subplots(figsize=(6, 4))
        ax.hist(xs, bins=50)
        ax.set_title(name)
        p = os.path.join(out_dir, f"dist_{name}.png")
        fig.savefig(p, dpi=80)
        plt.close(fig)
        files.append(p)
    if ok:
        fig, ax = plt.subplots(figsize=(6, 4))
        ax.scatter([r["prompt_tokens"] for r in ok], series["ttft"], s=4)
        ax.set_xlabel("prompt tokens")
        ax.set_ylabel("TTFT (s)")
        p = os.path.join(out_dir, "scatter_ttft_vs_prompt.png")
        fig.savefig(p, dpi=80)
        plt.close(fig)
        files.append(p)
    return files


def run(a) -> str:
    pname, text = load_profile(a.workload)
    cfg = apply_overrides(render(text, a.endpoint_url, a.model), a.overrides)
    ts = time.strftime("%Y%m%d-%H%M%S")
    ws = a.workspace or os.path.join(os.getcwd(), f"llmd-bench-{ts}")
    runner = os.path.join(ws, f"runner-{ts}")
    exp = f"{(a.spec or 'adhoc').replace('/', '_')}-{os.path.splitext(pname)[0]}-{a.harness}"
    res_dir = os.path.join(runner, "results", exp)
    os.makedirs(os.path.join(runner, "plan"), exist_ok=True)
    os.makedirs(res_dir, exist_ok=True)
    for d in (os.path.join(runner, "plan"), res_dir):
        with open(os.path.join(d, pname if pname.endswith(".yaml") else pname + ".yaml"), "w") as f:
            yaml.safe_dump(cfg, f, sort_keys=False)
    with open(os.path.join(res_dir, "config.yaml"), "w") as f:
        yaml.safe_dump({"spec": a.spec, "harness": a.harness, "endpoint_url": a.endpoint_url, "model": a.model,
                        "workload": pname, "overrides": a.overrides}, f, sort_keys=False)
    log = open(os.path.join(res_dir, "stdout.log"), "w")

    def say(msg):
        print(msg, flush=True)
        log.write(msg + "\n")
        log.flush()

    say(f"[benchmark] {pname} -> {a.endpoint_url} ({a.model}); results in {res_dir}")
    vocab = int(a.vocab)
    rep = asyncio.run(loadgen.run(cfg, vocab=vocab, seed=a.seed, records=True))
    for st in rep["stages"]:
        i = st["stage"]
        with open(os.path.join(res_dir, f"stage_{i}_lifecycle_metrics.json"), "w") as f:
            json.dump(st, f, indent=1)
        with open(os.path.join(res_dir, f"benchmark_report,_stage_{i}.yaml"), "w") as f:
            yaml.safe_dump(benchmark_report(st, cfg, i, a.model, a.harness), f, sort_keys=False)
        t = st["throughput"]
        say(f"[benchmark] stage {i} {st['config']}: {t['output_tokens_per_sec']:.1f} out tok/s, "
            f"{t['requests_per_sec']:.2f} req/s, TTFT p50 {st['latency']['time_to_first_token']['p50']}, "
            f"failures {st['requests']['failures']}")
    with open(os.path.join(res_dir, "summary_lifecycle_metrics.json"), "w") as f:
        json.dump(rep["summary"], f, indent=1)
    with open(os.path.join(res_dir, "benchmark_report,_summary.yaml"), "w") as f:
        yaml.safe_dump(benchmark_report(rep["summary"], cfg, None, a.model, a.harness), f, sort_keys=False)
    with open(os.path.join(res_dir, "per_request_lifecycle_metrics.json"), "w") as f:
        json.dump(rep["per_request"], f)
    if a.analyze:
        files = analyze(rep["per_request"], os.path.join(res_dir, "analysis", "distributions"))
        say(f"[benchmark] analysis: {len(files)} figures")
    log.close()
    return res_dir


def main(argv=None):
    p = argparse.ArgumentParser("llmd-benchmark")
    p.add_argument("--workspace", default=None)
    p.add_argument("--spec", default=None, help="guides/<name> (recorded in the report)")
    p.add_argument("--non-admin", action="store_true", help="accepted for CLI compatibility")
    sub = p.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--endpoint-url", required=True)
    r.add_argument("--model", required=True)
    r.add_argument("--workload", required=True)
    r.add_argument("--harness", default="inference-perf", choices=HARNESSES,
                   help="recorded in the report; the driver is the repo's load generator")
    r.add_argument("--gateway-class", default="epponly", help="accepted for CLI compatibility")
    r.add_argument("--namespace", default=None, help="accepted for CLI compatibility")
    r.add_argument("--overrides", default="")
    r.add_argument("--analyze", action="store_true")
    r.add_argument("--vocab", type=int, default=32000, help="token ids are drawn from [100, vocab - 100)")
    r.add_argument("--seed", type=int, default=0)
    sub.add_parser("list-workloads")
    a = p.parse_args(argv)
    if a.cmd == "list-workloads":
        print("\n".join(list_workloads()))
        return 0
    run(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
