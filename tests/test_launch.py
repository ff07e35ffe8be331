"""Single-node launcher plan (C40/C41): GPU assignment, TP packing, LWS env,
P/D roles with sidecars, router endpoints file."""
import os
import time

import yaml

from llmd_amd.launch import plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pd_topology_plan():
    with open(os.path.join(ROOT, "deploy/single-node/pd-70b-6p2d.yaml")) as f:
        topo = yaml.safe_load(f)
    specs, doc = plan(topo, "/tmp/w")
    eng = [s for s in specs if s.role in ("prefill", "decode")]
    assert [s.gpus for s in eng] == [[i] for i in range(8)]
    assert sum(s.role == "sidecar" for s in specs) == 2 and specs[-1].name == "router"
    pre = [s for s in eng if s.role == "prefill"]
    assert all("kv_producer" in " ".join(s.cmd) for s in pre)
    roles = [e["labels"]["llm-d.ai/role"] for e in doc["endpoints"]]
    assert roles == ["prefill"] * 6 + ["decode"] * 2
    assert [e["port"] for e in doc["endpoints"]][-2:] == [8400, 8401]  # decode via sidecar


def test_tp_packing_and_overflow():
    topo = {"model": "llama-3-70b", "gpus": 8,
            "roles": [{"name": "decode", "replicas": 2, "tp": 4, "port": 9000}]}
    specs, _ = plan(topo, "/tmp/w")
    assert [s.gpus for s in specs] == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert specs[0].env["LWS_GROUP_SIZE"] == "4" and "torch.distributed.run" in specs[0].cmd
    topo["roles"][0]["replicas"] = 3
    try:
        plan(topo, "/tmp/w")
        raise AssertionError("expected overflow")
    except ValueError:
        pass


def test_baseline_kv_events_labels():
    with open(os.path.join(ROOT, "deploy/single-node/optimized-baseline-8b.yaml")) as f:
        topo = yaml.safe_load(f)
    specs, doc = plan(topo, "/tmp/w")
    ports = [e["labels"]["llm-d.ai/kv-events-port"] for e in doc["endpoints"]]
    assert len(set(ports)) == 8
    assert all("--kv-events-config" in s.cmd for s in specs if s.role == "prefill-decode")


def test_deploy_values_and_router_configs_valid():
    import glob

    from llmd_amd.router.config import load_config

    files = glob.glob(os.path.join(ROOT, "deploy/**/*.yaml"), recursive=True)
    files = [f for f in files if "/templates/" not in f]
    assert len(files) >= 10
    n_cfg = 0
    for f in files:
        with open(f) as fh:
            doc = yaml.safe_load(fh)
        conf = ((doc or {}).get("router") or {})
        text = conf.get("pluginsConfig") or conf.get("config")
        if isinstance(text, str):
            load_config(text)
            n_cfg += 1
    assert n_cfg >= 4


def test_dashboards_reference_exported_metrics():
    import glob
    import json
    import re

    from llmd_amd.engine.metrics import EngineMetrics
    from llmd_amd.router.metrics import EPPMetrics

    names = set(re.findall(r"^# TYPE (\S+)", EngineMetrics("m", 16, 100).render().decode(), re.M))
    names |= set(re.findall(r"^# TYPE (\S+)", EPPMetrics().render().decode(), re.M))
    from llmd_amd.kvcache.offload import _XferStats

    names |= set(re.findall(r"^# TYPE (\S+)", "\n".join(_XferStats().render('model_name="m"')), re.M))
    import llmd_amd.kvcache.offload as off  # the tier's own gauges / counters (rendered per engine)

    names |= set(re.findall(r"# TYPE (vllm:[a-z_]+)", open(off.__file__).read()))
    names |= {"vllm:nixl_xfer_time_seconds", "vllm:nixl_bytes_transferred", "vllm:nixl_num_failed_transfers"}
    files = glob.glob(os.path.join(ROOT, "deploy/observability/grafana/dashboards/*.json"))
    assert len(files) == 6
    for f in files:
        for p in json.load(open(f))["panels"]:
            for t in p["targets"]:
                for m in re.findall(r"(vllm:[a-z0-9_]+|inference_[a-z0-9_]+|llm_d_[a-z0-9_]+)",
                                   re.sub(r"\{[^}]*\}", "", t["expr"])):  # metric names, not labels
                    base = re.sub(r"_(bucket|sum|count|total)$", "", m)
                    assert base in names or m in names, (f, m)


def test_router_extproc_mode_and_envoy_config():
    topo = {"model": "llama-3-8b", "gpus": 2, "roles": [{"name": "both", "replicas": 2}],
            "router": {"mode": "extproc", "grpc_port": 9102}}
    specs, _ = plan(topo, "/tmp/w")
    r = specs[-1]
    assert r.name == "router" and r.port == 9102 and "llmd_amd.router.extproc" in r.cmd
    with open(os.path.join(ROOT, "deploy/standalone/envoy-extproc.yaml")) as f:
        env = yaml.safe_load(f)
    hcm = env["static_resources"]["listeners"][0]["filter_chains"][0]["filters"][0]["typed_config"]
    ext = hcm["http_filters"][0]["typed_config"]
    assert ext["processing_mode"]["request_body_mode"] == "FULL_DUPLEX_STREAMED"
    cl = {c["name"]: c for c in env["static_resources"]["clusters"]}
    assert cl["picked_endpoint"]["original_dst_lb_config"]["http_header_name"] == "x-gateway-destination-endpoint"
    ep = cl["llmd_epp"]["load_assignment"]["endpoints"][0]["lb_endpoints"][0]["endpoint"]["address"]
    assert ep["socket_address"]["port_value"] == 9002


def test_cpu_opt125m_baseline_end_to_end(tmp_path):
    """The reference's CPU optimized-baseline config (OPT-125m on CPU engines,
    docker/Dockerfile.cpu): launcher -> 2 CPU engines + router -> completions
    served through the router."""
    import json
    import urllib.request

    from llmd_amd.launch import Launcher

    with open(os.path.join(ROOT, "deploy/single-node/optimized-baseline-opt125m-cpu.yaml")) as f:
        topo = yaml.safe_load(f)
    topo["router"]["port"] = 18310
    topo["roles"][0]["port"] = 18320
    specs, _ = plan(topo, str(tmp_path))
    eng = [s for s in specs if s.role == "prefill-decode"]
    assert len(eng) == 2 and all(s.gpus == [] and "--device" in s.cmd for s in eng)
    la = Launcher(topo, workdir=str(tmp_path)).start()
    try:
        assert la.wait_ready(timeout=300), open(tmp_path / "prefill-decode-0.log").read()[-3000:]
        body = json.dumps({"model": "facebook/opt-125m", "prompt": "the quick brown fox " * 20,
                           "max_tokens": 4}).encode()
        outs = []
        for _ in range(30):  # the router may need a scrape before it serves
            try:
                req = urllib.request.Request("http://127.0.0.1:18310/v1/completions", data=body,
                                             headers={"content-type": "application/json"})
                with urllib.request.urlopen(req, timeout=60) as r:
                    outs.append((json.loads(r.read()), r.status))
                if len(outs) == 2:
                    break
            except OSError:
                time.sleep(1.0)
        assert len(outs) == 2 and all(o["usage"]["completion_tokens"] == 4 for o, _ in outs)
    finally:
        la.stop()
