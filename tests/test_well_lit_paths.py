"""Single-node topologies of every reference well-lit path (guides/*):
deploy/single-node/*.yaml plan cleanly through the launcher (GPU packing,
DP ranks, services, router config validated by the EPP config loader), and a
CPU end-to-end run of the services path: tiny engines + router + latency
predictor + batch gateway started by the launcher, a batch job served through
the router, and the router's predicted-latency producer feeding the predictor
service (PREDICTION_SERVER_URL wired by the launcher)."""
import asyncio
import glob
import json
import os
import time
import urllib.request

import aiohttp
import yaml

from llmd_amd.launch import Launcher, plan
from llmd_amd.router.config import load_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GUIDES = {"optimized-baseline", "precise-prefix-cache-routing", "pd-70b", "wide-ep", "tiered-prefix-cache",
          "workload-autoscaling", "flow-control", "predicted-latency", "agentic-serving", "multimodal-e-pd",
          "batch-async"}


def test_every_guide_has_a_single_node_topology():
    files = sorted(glob.glob(os.path.join(ROOT, "deploy/single-node/*.yaml")))
    names = {os.path.basename(f) for f in files}
    for g in GUIDES:
        assert any(n.startswith(g) for n in names), g
    for f in files:
        topo = yaml.safe_load(open(f))
        specs, doc = plan(topo, "<workdir>")
        conf = (topo.get("router") or {}).get("config")
        if conf:
            load_config(conf)
        gpus = [g for s in specs for g in s.gpus]
        assert len(gpus) == len(set(gpus)) and all(0 <= g < int(topo.get("gpus", 8)) for g in gpus), f
        if "wide-ep" in f:
            assert [e["port"] for e in doc["endpoints"]] == list(range(8200, 8208))
            assert "--nproc-per-node=8" in specs[0].cmd and "--data-parallel-size" in specs[0].cmd
        if "predicted-latency" in f:
            assert specs[-1].env["PREDICTION_SERVER_URL"].endswith(":8100")


def _post(url, body, timeout=60):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), headers={"content-type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read())


def test_services_end_to_end_cpu(tmp_path):
    topo = {"model": "tiny-llama", "device": "cpu",
            "services": [{"type": "predictor", "port": 18451}, {"type": "batch-gateway", "port": 18452}],
            "router": {"port": 18450, "config": """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: approx-prefix-cache-producer
- type: predicted-latency-producer
- type: queue-scorer
- type: prefix-cache-scorer
- type: max-score-picker
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: predicted-latency-producer
  - pluginRef: queue-scorer
  - pluginRef: prefix-cache-scorer
  - pluginRef: max-score-picker
"""},
            "roles": [{"name": "prefill-decode", "replicas": 2, "port": 18460,
                       "args": ["--max-num-seqs", "8", "--max-model-len", "512", "--num-gpu-blocks-override", "64",
                                "--block-size", "16", "--enforce-eager"]}]}
    la = Launcher(topo, workdir=str(tmp_path)).start()
    try:
        logs = lambda: {p: open(p).read()[-1500:] for p in glob.glob(str(tmp_path / "*.log"))}  # noqa: E731
        assert la.wait_ready(timeout=300), logs()
        # direct traffic through the router: the producer streams training samples to the predictor
        outs = []
        for i in range(40):
            try:
                outs.append(_post("http://127.0.0.1:18450/v1/completions",
                                  {"model": "tiny-llama", "prompt": f"request {i} " * 10, "max_tokens": 4}))
            except OSError:
                time.sleep(0.5)
        assert len(outs) >= 30 and all(o["usage"]["completion_tokens"] == 4 for o in outs)

        async def batch():
            base = "http://127.0.0.1:18452"
            data = "\n".join(json.dumps({"custom_id": f"c{i}", "method": "POST", "url": "/v1/completions",
                                         "body": {"model": "tiny-llama", "prompt": f"batch {i}", "max_tokens": 3}})
                             for i in range(6)).encode()
            async with aiohttp.ClientSession() as s:
                fd = aiohttp.FormData()
                fd.add_field("purpose", "batch")
                fd.add_field("file", data, filename="in.jsonl")
                async with s.post(base + "/v1/files", data=fd) as r:
                    f = await r.json()
                async with s.post(base + "/v1/batches", json={"input_file_id": f["id"], "endpoint": "/v1/completions",
                                                              "completion_window": "24h"}) as r:
                    b = await r.json()
                t0 = time.time()
                while time.time() - t0 < 120:
                    async with s.get(f"{base}/v1/batches/{b['id']}") as r:
                        b = await r.json()
                    if b["status"] in ("completed", "failed"):
                        break
                    await asyncio.sleep(0.2)
                async with s.get(f"{base}/v1/files/{b['output_file_id']}/content") as r:
                    lines = [json.loads(x) for x in (await r.text()).splitlines() if x.strip()]
                return b, lines

        b, lines = asyncio.run(batch())
        assert b["status"] == "completed" and b["request_counts"]["completed"] == 6, b
        assert all(x["response"]["status_code"] == 200 for x in lines)
        # the predictor service received the router's samples
        with urllib.request.urlopen("http://127.0.0.1:18451/metrics", timeout=5) as r:
            m = r.read().decode()
        samples = [line for line in m.splitlines() if line.startswith("latency_predictor_ttft_samples")]
        assert samples and float(samples[0].split()[-1]) > 0, m[-2000:]
    finally:
        la.stop()
