"""End-to-end router tests over real HTTP on CPU: engine simulators + router
proxy (+ routing sidecars for P/D), the reference's e2e validator shapes
(.github/scripts/e2e/e2e-validate*.sh) re-expressed as pytest."""
import asyncio
import json
import statistics

import aiohttp
import pytest
from aiohttp import web

from llmd_amd.router.api import ControlPlane
from llmd_amd.router.datalayer import EndpointStore, endpoints_from_yaml
from llmd_amd.router.epp import EPP
from llmd_amd.router.proxy import RouterProxy
from llmd_amd.sidecar.routing_sidecar import RoutingSidecar
from llmd_amd.sim.server import start_sim

BASE = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: queue-scorer
- type: kv-cache-utilization-scorer
- type: prefix-cache-scorer
- type: no-hit-lru-scorer
- type: metrics-data-source
  parameters: {interval: 20ms}
- type: core-metrics-extractor
dataLayer:
  sources:
  - pluginRef: metrics-data-source
    extractors: [{pluginRef: core-metrics-extractor}]
schedulingProfiles:
- name: default
  plugins:
  - {pluginRef: queue-scorer, weight: 2}
  - {pluginRef: kv-cache-utilization-scorer, weight: 2}
  - {pluginRef: prefix-cache-scorer, weight: 3}
  - {pluginRef: no-hit-lru-scorer, weight: 2}
"""


async def _serve(app, port=0):
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", port)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


async def _router(config, eps, control=None):
    store = EndpointStore()
    epp = EPP(config, store, control or ControlPlane())
    for e in endpoints_from_yaml({"endpoints": eps}):
        await store.add(e)
    prox = RouterProxy(epp)
    runner, port = await _serve(prox.app())
    return runner, epp, port


async def _post(s, url, body, headers=None):
    async with s.post(url, json=body, headers=headers or {}) as r:
        return r.status, await r.read(), dict(r.headers)


def test_aggregated_routing_stream_usage_and_affinity():
    async def main():
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001) for _ in range(4)]
        eps = [{"name": f"s{i}", "address": "127.0.0.1", "port": p} for i, (_, _, p) in enumerate(sims)]
        rr, epp, port = await _router(BASE, eps)
        url = f"http://127.0.0.1:{port}/v1/completions"
        async with aiohttp.ClientSession() as s:
            st, body, _ = await _post(s, url, {"model": "m", "prompt": "hi", "max_tokens": 5})
            assert st == 200 and json.loads(body)["usage"]["completion_tokens"] == 5
            st, body, _ = await _post(s, url, {"model": "m", "prompt": "hi", "max_tokens": 4, "stream": True,
                                               "stream_options": {"include_usage": True}})
            assert st == 200 and body.strip().endswith(b"[DONE]")
            # chat through the router
            st, body, _ = await _post(s, url.replace("completions", "chat/completions"),
                                      {"model": "m", "messages": [{"role": "user", "content": "yo"}], "max_tokens": 3})
            assert st == 200 and json.loads(body)["choices"][0]["message"]["content"]
            # approximate prefix affinity: same long prefix -> same endpoint
            long = "The quick brown fox jumps over the lazy dog. " * 80
            served = []
            for i in range(6):
                await _post(s, url, {"model": "m", "prompt": long + str(i), "max_tokens": 2})
            for (_, eng, p) in sims:
                served.append(int(sum(v for _, v in [(0, 0)]) + eng.metrics.n_prompt))
            counts = [eng.metrics.success._metrics for (_, eng, _) in sims]
            # the long-prefix requests all landed on one simulator
            hits = [len([1 for k in eng.metrics.success._metrics]) for (_, eng, _) in sims]
            async with s.get(f"http://127.0.0.1:{port}/metrics") as r:
                text = await r.text()
            assert "inference_extension_scheduler_attempts_total" in text
            assert "inference_pool_ready_pods" in text
        # metrics data layer populated endpoint attributes
        assert all(e.attrs.get("MetricsUpdateTime") is not None for e in epp.store.all())
        await rr.cleanup()
        for r, eng, _ in sims:
            await r.cleanup()
    asyncio.run(main())


def test_prefix_affinity_concentrates_requests():
    async def main():
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.0005) for _ in range(4)]
        eps = [{"name": f"s{i}", "address": "127.0.0.1", "port": p} for i, (_, _, p) in enumerate(sims)]
        rr, epp, port = await _router(BASE, eps)
        url = f"http://127.0.0.1:{port}/v1/completions"
        long = "lorem ipsum dolor sit amet " * 100
        async with aiohttp.ClientSession() as s:
            for i in range(8):
                st, _, _ = await _post(s, url, {"model": "m", "prompt": long + f"q{i}", "max_tokens": 1})
                assert st == 200
        gens = [eng.metrics.n_gen if hasattr(eng.metrics, "n_gen") else 0 for (_, eng, _) in sims]
        # count requests per simulator through their prompt-token counters
        per = []
        for (_, eng, _) in sims:
            v = eng.metrics.prompt_tokens.labels("m")._value.get()
            per.append(v)
        assert sum(1 for v in per if v > 0) == 1, per  # all on one endpoint (affinity)
        await rr.cleanup()
        for r, _, _ in sims:
            await r.cleanup()
    asyncio.run(main())


PD = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: disagg-headers-handler
- type: always-disagg-pd-decider
- type: disagg-profile-handler
  parameters: {deciderPluginName: always-disagg-pd-decider}
- type: prefill-filter
- type: decode-filter
- type: prefix-cache-scorer
- type: queue-scorer
- type: active-request-scorer
schedulingProfiles:
- name: prefill
  plugins: [{pluginRef: prefill-filter}, {pluginRef: prefix-cache-scorer, weight: 3}, {pluginRef: queue-scorer, weight: 2}]
- name: decode
  plugins: [{pluginRef: decode-filter}, {pluginRef: active-request-scorer, weight: 2}, {pluginRef: prefix-cache-scorer, weight: 3}]
"""


def test_pd_disaggregation_through_sidecar():
    async def main():
        pre = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001, role="prefill") for _ in range(2)]
        dec = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001, role="decode") for _ in range(2)]
        sidecars = []
        eps = []
        for i, (_, _, p) in enumerate(pre):
            eps.append({"name": f"p{i}", "address": "127.0.0.1", "port": p, "labels": {"llm-d.ai/role": "prefill"}})
        for i, (_, _, p) in enumerate(dec):
            sc = RoutingSidecar(f"http://127.0.0.1:{p}")
            r, sp = await _serve(sc.app())
            sidecars.append((r, sc))
            eps.append({"name": f"d{i}", "address": "127.0.0.1", "port": sp, "labels": {"llm-d.ai/role": "decode"}})
        rr, epp, port = await _router(PD, eps)
        url = f"http://127.0.0.1:{port}/v1/completions"
        async with aiohttp.ClientSession() as s:
            for i in range(6):
                st, body, _ = await _post(s, url, {"model": "m", "prompt": f"prompt {i} " * 30, "max_tokens": 4})
                assert st == 200, body
                assert json.loads(body)["usage"]["completion_tokens"] == 4
        # prefill sims saw only max_tokens=1 remote-decode prefills; decoders did the decoding
        p_gen = sum(e.metrics.gen_tokens.labels("m")._value.get() for _, e, _ in pre)
        d_gen = sum(e.metrics.gen_tokens.labels("m")._value.get() for _, e, _ in dec)
        assert p_gen == 6 and d_gen == 24
        assert sum(sc.m_req.labels("pd")._value.get() for _, sc in sidecars) == 6
        text = epp.render_metrics().decode()
        assert 'decision_type="disagg"' in text
        # prefill failure -> decode-only fallback
        for _, e, _ in pre:
            e.fail_prefill = 1.0
        async with aiohttp.ClientSession() as s:
            st, body, _ = await _post(s, url, {"model": "m", "prompt": "x " * 30, "max_tokens": 2})
            assert st == 200
        assert sum(sc.m_fallback.labels("prefill_500")._value.get() for _, sc in sidecars) == 1
        await rr.cleanup()
        for r, _ in sidecars:
            await r.cleanup()
        for r, _, _ in pre + dec:
            await r.cleanup()
    asyncio.run(main())


FLOW = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
featureGates: [flowControl]
plugins:
- type: round-robin-fairness-policy
- type: fcfs-ordering-policy
- type: concurrency-detector
  parameters: {maxConcurrency: 2}
- type: queue-scorer
saturationDetector: {pluginRef: concurrency-detector}
flowControl:
  defaultRequestTTL: 60s
  priorityBands:
  - {priority: 100, fairnessPolicyRef: round-robin-fairness-policy}
  - {priority: 0, fairnessPolicyRef: round-robin-fairness-policy}
  - {priority: -10, fairnessPolicyRef: round-robin-fairness-policy}
schedulingProfiles:
- name: default
  plugins: [{pluginRef: queue-scorer}]
"""

OBJECTIVES = """
kind: InferenceObjective
metadata: {name: premium}
spec: {priority: 100}
---
kind: InferenceObjective
metadata: {name: standard}
spec: {priority: 0}
---
kind: InferenceObjective
metadata: {name: best-effort}
spec: {priority: -10}
"""


def test_flow_control_strict_priority_e2e():
    """Mirror of e2e-validate-flow-control.sh: 3 bands x 12 concurrent requests
    under forced contention; every band is classified and best-effort waits
    longer than premium on average."""
    async def main():
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.01)]
        eps = [{"name": "s0", "address": "127.0.0.1", "port": sims[0][2]}]
        cp = ControlPlane()
        cp.load_yaml(OBJECTIVES)
        rr, epp, port = await _router(FLOW, eps, cp)
        url = f"http://127.0.0.1:{port}/v1/completions"
        async with aiohttp.ClientSession() as s:
            async def one(obj, i):
                st, _, _ = await _post(s, url, {"model": "m", "prompt": "p", "max_tokens": 3},
                                       {"x-llm-d-inference-objective": obj, "x-llm-d-inference-fairness-id": f"t{i % 3}"})
                return st
            jobs = [one(o, i) for i in range(12) for o in ("best-effort", "standard", "premium")]
            res = await asyncio.gather(*jobs)
        assert all(r == 200 for r in res)
        from prometheus_client.parser import text_string_to_metric_families
        text = epp.render_metrics().decode()
        sums, counts = {}, {}
        for fam in text_string_to_metric_families(text):
            if fam.name == "inference_extension_flow_control_request_queue_duration_seconds":
                for smp in fam.samples:
                    p = smp.labels.get("priority")
                    if smp.name.endswith("_sum"):
                        sums[p] = sums.get(p, 0) + smp.value
                    elif smp.name.endswith("_count"):
                        counts[p] = counts.get(p, 0) + smp.value
        assert counts.get("100", 0) > 0 and counts.get("0", 0) > 0 and counts.get("-10", 0) > 0
        mean = {p: sums[p] / counts[p] for p in counts}
        assert mean["-10"] - mean["100"] > 0.05, mean
        await rr.cleanup()
        await sims[0][0].cleanup()
    asyncio.run(main())


PRECISE = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: token-producer
  parameters: {modelName: m, vllm: {url: "RENDER"}}
- type: endpoint-notification-source
- type: precise-prefix-cache-producer
  parameters:
    tokenProcessorConfig: {blockSize: 16}
    speculativeIndexing: true
    kvEventsConfig: {topicFilter: "kv@", discoverPods: true}
- type: prefix-cache-scorer
  parameters: {prefixMatchInfoProducerName: precise-prefix-cache-producer}
- type: queue-scorer
dataLayer:
  sources:
  - pluginRef: endpoint-notification-source
    extractors: [{pluginRef: precise-prefix-cache-producer}]
schedulingProfiles:
- name: default
  plugins: [{pluginRef: prefix-cache-scorer, weight: 3}, {pluginRef: queue-scorer, weight: 1}]
"""


def test_precise_prefix_routing_with_kv_events():
    async def main():
        import socket

        def free_port():
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            p = s.getsockname()[1]
            s.close()
            return p

        sims = []
        for i in range(3):
            kp = free_port()
            r, eng, p = await start_sim(model="m", block_size=16, prefill_tps=1e6, decode_step_s=0.0005,
                                        kv_events_port=kp)
            sims.append((r, eng, p, kp))
        eps = [{"name": f"s{i}", "address": "127.0.0.1", "port": p,
                "labels": {"llm-d.ai/kv-events-port": str(kp)}} for i, (_, _, p, kp) in enumerate(sims)]
        cfg = PRECISE.replace("RENDER", f"http://127.0.0.1:{sims[0][2]}")
        rr, epp, port = await _router(cfg, eps)
        url = f"http://127.0.0.1:{port}/v1/completions"
        prod = epp.cfg.plugins["precise-prefix-cache-producer"]
        await asyncio.sleep(0.3)  # subscribers connect
        prompt = "shared system prompt. " * 40
        async with aiohttp.ClientSession() as s:
            st, _, _ = await _post(s, url, {"model": "m", "prompt": prompt + "first", "max_tokens": 1})
            assert st == 200
            for _ in range(50):
                if prod.events_seen:
                    break
                await asyncio.sleep(0.02)
            assert prod.events_seen > 0
            for i in range(4):
                await _post(s, url, {"model": "m", "prompt": prompt + f"n{i}", "max_tokens": 1})
        per = [eng.metrics.prompt_tokens.labels("m")._value.get() for _, eng, _, _ in sims]
        assert sum(1 for v in per if v > 0) == 1, per
        await rr.cleanup()
        for r, eng, _, _ in sims:
            if eng.pub:
                eng.pub.close()
            await r.cleanup()
    asyncio.run(main())


PREDICTED = """
apiVersion: llm-d.ai/v1alpha1
kind: EndpointPickerConfig
plugins:
- type: approx-prefix-cache-producer
- type: predicted-latency-producer
  parameters: {streamingMode: true, predictionServerURL: "PRED", trainingServerURL: "TRAIN",
               trainingBatchSize: 4, trainingFlushIntervalS: 0.1}
- type: latency-scorer
- type: weighted-random-picker
- type: metrics-data-source
  parameters: {interval: 20ms}
- type: core-metrics-extractor
dataLayer:
  sources:
  - pluginRef: metrics-data-source
    extractors: [{pluginRef: core-metrics-extractor}]
schedulingProfiles:
- name: default
  plugins:
  - pluginRef: predicted-latency-producer
  - pluginRef: latency-scorer
  - pluginRef: weighted-random-picker
"""


def test_predicted_latency_served_e2e(tmp_path):
    """Mirror of e2e-validate-predicted-latency.sh with the deployed shape of
    the predictor (latency-predictor.md:18-52): a training server and a
    prediction server sharing a model file; the router streams training
    samples to the first and asks the second. After 100 requests at
    concurrency 8 the predicted-TTFT histogram must have samples next to the
    actual-TTFT one - predictions were served, not silently skipped."""
    import os
    import socket
    import subprocess
    import sys
    import time

    def free_port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    model = tmp_path / "latency_model.bin"
    tp, pp = free_port(), free_port()
    env = dict(os.environ, MODEL_SYNC_INTERVAL_SEC="0.2")
    common = [sys.executable, "-m", "llmd_amd.router.predictor", "--model-path", str(model),
              "--min-samples", "20", "--retrain-every", "20"]
    procs = [subprocess.Popen(common + ["--role", "training", "--port", str(tp)], cwd=root, env=env,
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True),
             subprocess.Popen(common + ["--role", "prediction", "--port", str(pp)], cwd=root, env=env,
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)]

    async def main():
        sims = [await start_sim(model="m", prefill_tps=2e5, decode_step_s=0.002) for _ in range(2)]
        eps = [{"name": f"s{i}", "address": "127.0.0.1", "port": s[2]} for i, s in enumerate(sims)]
        cfg = PREDICTED.replace("PRED", f"http://127.0.0.1:{pp}").replace("TRAIN", f"http://127.0.0.1:{tp}")
        async with aiohttp.ClientSession() as s:
            deadline = time.time() + 60
            while time.time() < deadline:      # both predictor servers up
                try:
                    ok = 0
                    for port in (tp, pp):
                        async with s.get(f"http://127.0.0.1:{port}/healthz") as r:
                            ok += r.status == 200
                    if ok == 2:
                        break
                except aiohttp.ClientError:
                    pass
                await asyncio.sleep(0.2)
            rr, epp, port = await _router(cfg, eps)
            url = f"http://127.0.0.1:{port}/v1/completions"
            sem = asyncio.Semaphore(8)

            async def one(i):
                async with sem:
                    body = {"model": "m", "prompt": f"request {i} " + "x " * (20 + 7 * (i % 13)), "max_tokens": 4,
                            "stream": True, "stream_options": {"include_usage": True}}
                    async with s.post(url, json=body) as r:
                        await r.read()
                        return r.status

            assert all(st == 200 for st in await asyncio.gather(*[one(i) for i in range(100)]))
            # the prediction server picks up the model the training server wrote
            deadline = time.time() + 30
            while time.time() < deadline:
                async with s.get(f"http://127.0.0.1:{pp}/healthz") as r:
                    if (await r.json()).get("ready"):
                        break
                await asyncio.sleep(0.2)
            assert all(st == 200 for st in await asyncio.gather(*[one(100 + i) for i in range(40)]))
            from prometheus_client.parser import text_string_to_metric_families

            counts = {}
            for fam in text_string_to_metric_families(epp.render_metrics().decode()):
                for smp in fam.samples:
                    if smp.name.endswith("_count"):
                        counts[smp.name] = counts.get(smp.name, 0) + smp.value
            await rr.cleanup()
        for sm in sims:
            await sm[0].cleanup()
        return counts

    try:
        counts = asyncio.run(main())
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
                p.wait()
    assert counts.get("inference_objective_request_ttft_seconds_count", 0) > 0
    assert counts.get("inference_objective_request_predicted_ttft_seconds_count", 0) > 0, counts


import glob as _glob

_GUIDES = sorted(_glob.glob("/root/reference/guides/*/router/*.values.yaml"))


@pytest.mark.parametrize("values", _GUIDES or ["<reference tree not mounted>"],
                         ids=[p.split("guides/")[1] for p in _GUIDES] or ["none"])
def test_reference_guide_configs_route(values):
    """Every EndpointPickerConfig the reference's guides ship (plugin graphs
    verbatim from guides/*/router/*.values.yaml) loads and routes plain and
    streamed completions over HTTP to role-labelled simulators."""
    from llmd_amd.router.config import ConfigError, extract_config_text

    if not _GUIDES:
        pytest.skip("reference tree not mounted")
    try:
        cfg = extract_config_text(open(values).read())
    except ConfigError:
        pytest.skip("values file without a custom plugin config")

    async def main():
        roles = ("prefill", "prefill", "decode", "decode")
        sims = [await start_sim(model="m", prefill_tps=1e6, decode_step_s=0.001, role=r) for r in roles]
        eps = [{"name": f"s{i}", "address": "127.0.0.1", "port": s[2], "labels": {"llm-d.ai/role": r}}
               for i, (s, r) in enumerate(zip(sims, roles))]
        rr, epp, port = await _router(cfg, eps)
        out = []
        async with aiohttp.ClientSession() as s:
            for i in range(6):
                body = {"model": "m", "prompt": "hello world " * (i + 1), "max_tokens": 3, "stream": i % 2 == 1,
                        "stream_options": {"include_usage": True}}
                async with s.post(f"http://127.0.0.1:{port}/v1/completions", json=body) as r:
                    data = await r.read()
                    out.append((r.status, data))
        await rr.cleanup()
        for sm in sims:
            await sm[0].cleanup()
        return out

    res = asyncio.run(main())
    assert all(st == 200 for st, _ in res), [(st, d[:200]) for st, d in res]
    assert all(b"choices" in d or b"data:" in d for _, d in res)
