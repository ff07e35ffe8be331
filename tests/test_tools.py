"""Operator tools (C37-C39): tuning-wizard math, calibration, healthcheck and
the load generator, against the engine simulator over HTTP on CPU."""
import asyncio
import io
import math
import threading

import pytest

from llmd_amd.sim.server import start_sim
from llmd_amd.tools import healthcheck, loadgen, tuning


class SimThread:
    """Simulator on its own event-loop thread (for the synchronous tools)."""

    def __init__(self, **kw):
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        self.kw = kw
        threading.Thread(target=self._run, daemon=True).start()
        self.ready.wait(10)

    def _run(self):
        asyncio.set_event_loop(self.loop)
        self.runner, self.eng, self.port = self.loop.run_until_complete(start_sim(**self.kw))
        self.ready.set()
        self.loop.run_forever()

    def close(self):
        asyncio.run_coroutine_threadsafe(self.runner.cleanup(), self.loop).result(5)
        self.loop.call_soon_threadsafe(self.loop.stop)


@pytest.fixture(scope="module")
def sim():
    s = SimThread(model="m", prefill_tps=200000.0, decode_step_s=0.001)
    yield s
    s.close()


def test_tuning_math():
    assert tuning.compute_limit(10.0, 2.5) == 25
    n, isl, cv = tuning.memory_limit(1000, 64, efficiency=1.0, isl_mean=1000, osl_mean=200)
    mu = 1000 + 100
    sigma = math.sqrt(200 ** 2 / 12)
    # N*mu + z*sqrt(N)*sigma <= tokens at the solution, violated at N+2
    assert n * mu + 2.33 * math.sqrt(n) * sigma <= 64000
    assert (n + 2) * mu + 2.33 * math.sqrt(n + 2) * sigma > 64000
    n2, isl2, _ = tuning.memory_limit(1000, 64, efficiency=1.0, shared_prefix=500, isl_mean=1000, osl_mean=200)
    assert isl2 == 500 and n2 > n  # prefix caching frees the shared part
    assert tuning.lookahead_buffer(100, 8192, 1000) == 9
    assert tuning.lookahead_buffer(20, 8192, 100) == 3  # capped at 15%
    r = tuning.recommend(10.0, 2.5, 1000, 64, 8192, isl_mean=1000, osl_mean=200)
    assert r.active_batch == min(25, r.memory_limit) and r.max_concurrency == r.active_batch + r.lookahead_buffer
    assert "compute" in r.bottleneck and r.warnings  # N < 30 warning


def test_calibrate_and_healthcheck(sim):
    ep = f"http://127.0.0.1:{sim.port}"
    out = io.StringIO()
    res = tuning.calibrate(ep, "m", chunk=2000, warmup=1, measurements=3, out=out)
    assert "PEAK_PREFILL_THROUGHPUT=" in out.getvalue() and res["peak_prefill_throughput"] > 0
    rep = healthcheck.healthcheck(ep, max_latency_ms=5000)
    assert rep["status"] == "pass" and rep["model"] == "m" and rep["checks"]["inference"]["path"] == "/v1/completions"
    rep = healthcheck.healthcheck(ep, api_mode="chat")
    assert rep["status"] == "pass"
    bad = healthcheck.healthcheck("http://127.0.0.1:1", timeout=1)
    assert bad["status"] == "fail" and bad["checks"]["health"]["status"] == "warn"
    assert healthcheck.main(["-e", ep, "--output", "json"]) == 0


def test_loadgen_random_and_shared_prefix(sim):
    base = f"http://127.0.0.1:{sim.port}"
    cfg = {"load": {"type": "poisson", "stages": [{"rate": 40, "duration": 0.5}]},
           "server": {"base_url": base, "model_name": "m"},
           "data": {"type": "random", "input_distribution": {"mean": 64, "std": 8, "min": 32, "max": 96},
                    "output_distribution": {"mean": 8}}}
    rep = asyncio.run(loadgen.run(cfg, vocab=1000))
    s = rep["summary"]
    assert s["requests"]["total"] > 5 and s["requests"]["failures"] == 0
    assert s["latency"]["time_to_first_token"]["p50"] > 0 and s["throughput"]["output_tokens_per_sec"] > 0
    assert s["requests"]["output_length"]["mean"] == 8
    cfg2 = {"load": {"type": "concurrent", "stages": [{"concurrency": 4, "num_requests": 12}]},
            "server": {"base_url": base, "model_name": "m"},
            "data": {"type": "shared_prefix", "shared_prefix": {
                "num_groups": 2, "num_prompts_per_group": 3, "system_prompt_len": 64, "question_len": 16,
                "output_len": 4, "enable_multi_turn_chat": True}}}
    rep2 = asyncio.run(loadgen.run(cfg2, vocab=1000))
    st = rep2["stages"][0]
    assert st["requests"]["total"] == 12 and st["requests"]["failures"] == 0
    # multi-turn: second-round prompts carry the previous turn
    assert st["requests"]["input_length"]["max"] > 64 + 16


def test_benchmark_cli_workspace_and_reports(sim, tmp_path):
    """llmdbenchmark-style run against the simulator: every shipped profile
    renders; a shared-prefix ladder (overridden to 2 short stages) writes the
    reference's results layout with per-stage / summary / per-request files
    and cross-harness benchmark reports."""
    import json as _json

    import yaml as _yaml

    from llmd_amd.tools import benchmark

    names = benchmark.list_workloads()
    assert {"sanity_random.yaml", "shared_prefix_synthetic.yaml", "guide_optimized-baseline_1.yaml",
            "guide_pd-disaggregation_1.yaml"} <= set(names)
    for n in names:
        cfg = benchmark.render(benchmark.load_profile(n)[1], "http://x:1", "m")
        assert cfg["server"]["base_url"] == "http://x:1" and cfg["server"]["model_name"] == "m"
        assert cfg["load"]["stages"] and cfg["data"]["type"] in ("random", "shared_prefix")
    ov = benchmark.apply_overrides({"load": {"stages": [{"rate": 1}]}}, "load.stages.0.rate=5,data.x.y=true")
    assert ov == {"load": {"stages": [{"rate": 5}]}, "data": {"x": {"y": True}}}
    rc = benchmark.main(["--workspace", str(tmp_path), "--spec", "guides/optimized-baseline", "run",
                         "--endpoint-url", f"http://127.0.0.1:{sim.port}", "--model", "m",
                         "--workload", "shared_prefix_synthetic_short.yaml", "--vocab", "1000", "--analyze",
                         "--overrides", "load.stages=[{rate: 20, duration: 1}, {rate: 40, duration: 1}],"
                                        "data.shared_prefix.output_len=8"])
    assert rc == 0
    (runner,) = list(tmp_path.glob("runner-*"))
    (res,) = list((runner / "results").iterdir())
    files = {p.name for p in res.iterdir()}
    assert {"stage_0_lifecycle_metrics.json", "stage_1_lifecycle_metrics.json", "summary_lifecycle_metrics.json",
            "per_request_lifecycle_metrics.json", "benchmark_report,_stage_0.yaml", "benchmark_report,_stage_1.yaml",
            "config.yaml", "stdout.log", "analysis"} <= files
    rep = _yaml.safe_load((res / "benchmark_report,_stage_1.yaml").read_text())
    assert rep["scenario"]["load"]["config"]["rate"] == 40
    assert rep["metrics"]["requests"]["failures"] == 0 and rep["metrics"]["throughput"]["output_tokens_per_sec"] > 0
    per = _json.loads((res / "per_request_lifecycle_metrics.json").read_text())
    assert len(per) == rep["metrics"]["requests"]["total"] + _yaml.safe_load(
        (res / "benchmark_report,_stage_0.yaml").read_text())["metrics"]["requests"]["total"]
    assert all(r["output_tokens"] == 8 for r in per)
    assert list((res / "analysis" / "distributions").glob("dist_ttft.png"))
