"""Workload Variant Autoscaler controller for one node (the
reconcile loop of docs/architecture/advanced/autoscaling/wva.md:5-10,140-205 and
guides/workload-autoscaling/README.wva.md).

The reference WVA is a Kubernetes controller: it reads VariantAutoscaling
objects, queries vLLM metrics from Prometheus plus the EPP flow-control queue,
runs Analyzer -> Optimizer -> Enforcer (``wva.WVAEngine``) and publishes
``wva_desired_replicas`` for an HPA/KEDA to act on. On one 8xMI355X host there
is no Deployment to scale, so this controller closes the loop itself:

* ``variantAutoscalings`` - the VA objects verbatim (``llmd.ai/v1alpha1``,
  ``spec: {modelID, minReplicas, maxReplicas, variantCost, scaleTargetRef}``)
  plus a ``launch`` block per variant (the engine recipe the scale target would
  name: model, tp, portBase, args);
* every ``interval`` the controller scrapes each replica's ``/metrics``
  (``vllm:kv_cache_usage_perc``, ``vllm:num_requests_waiting`` /
  ``running``, ``vllm:cache_config_info``) and the router's
  ``inference_extension_flow_control_queue_size``, runs the engine and
  actuates through ``wva.ProcessActuator`` (engine processes on free GPUs);
* ready replicas are written to the router's file-discovery ``endpoints.yaml``
  (atomic rename; the router watches it), so a replica receives traffic once
  it answers ``/health`` and stops receiving it before it is stopped;
* a 100 ms fast loop runs scale-from-zero from the EPP queue (wva.md:197-201);
* ``/metrics`` exports ``wva_desired_replicas`` / ``wva_current_replicas`` /
  ``wva_desired_ratio`` labelled like the reference (``variant_name``,
  ``exported_namespace``, ``model_id``), for an HPA or for dashboards.

  python -m llmd_amd.autoscale.controller --config wva.yaml
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import threading
import time
import urllib.request
from typing import Optional

import yaml

from llmd_amd.router.datalayer import parse_prometheus

from .wva import ProcessActuator, ReplicaMetrics, Variant, WVAEngine, _dur

log = logging.getLogger("llmd.wva")
PY = sys.executable


def _get(url: str, timeout: float = 1.0) -> Optional[str]:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.read().decode()
    except OSError:
        return None


def _first(m: dict, name: str, default: float = 0.0) -> float:
    vals = m.get(name)
    return float(vals[0][1]) if vals else default


class WVAController:
    def __init__(self, cfg: dict, launch_cmd=None):
        self.cfg = cfg
        self.interval = _dur(cfg.get("interval", "30s"))
        self.fast_interval = float(cfg.get("fastInterval", 0.1))
        self.epp_metrics_url = cfg.get("eppMetricsUrl")
        self.endpoints_file = cfg.get("endpointsFile")
        self.namespace = cfg.get("namespace", "default")
        self.variants: dict[str, Variant] = {}
        self.launch: dict[str, dict] = {}
        for va in cfg.get("variantAutoscalings", []):
            spec = va.get("spec", {})
            name = va["metadata"]["name"]
            if int(spec.get("minReplicas", 1)) > int(spec.get("maxReplicas", 2)):
                raise ValueError(f"VariantAutoscaling {name}: minReplicas > maxReplicas")
            ln = dict(va.get("launch") or {})
            self.launch[name] = ln
            self.variants[name] = Variant(name=name, model_id=spec["modelID"],
                                          min_replicas=int(spec.get("minReplicas", 1)),
                                          max_replicas=int(spec.get("maxReplicas", 2)),
                                          cost=float(spec.get("variantCost", "10.0")),
                                          gpus_per_replica=int(ln.get("tp", 1)) if not ln.get("cpu") else 0)
        self._launch_cmd = launch_cmd or self._engine_cmd
        self.actuator = ProcessActuator(int(cfg.get("gpus", 8)), self._launch, env=cfg.get("env") or {})
        self.engine = WVAEngine(cfg.get("scalingConfig") or {}, actuator=None,
                                gpu_budget=int(cfg.get("gpus", 8)))
        self.retention = _dur((cfg.get("scalingConfig") or {}).get("retention_period", "10m"))
        self.last_activity: dict[str, float] = {}
        self.lock = threading.Lock()
        self.stop_ev = threading.Event()

    # ------------------------------------------------------------ actuation
    def _engine_cmd(self, v: Variant, ln: dict, port: int) -> list[str]:
        tp = int(ln.get("tp", 1))
        server = ["-m", "llmd_amd.serving.api_server", "--model", ln.get("model", v.model_id), "--port", str(port),
                  "--tensor-parallel-size", str(tp)] + (["--device", "cpu"] if ln.get("cpu") else []) + \
            [str(a) for a in ln.get("args", [])]
        if tp > 1:
            return [PY, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={tp}",
                    "--master-addr=127.0.0.1", f"--master-port={29700 + port % 1000}"] + server
        return [PY] + server

    def _launch(self, v: Variant, gpus: list[int], idx: int) -> list[str]:
        ln = self.launch[v.name]
        # the lowest port of the variant's range that no running replica holds (replicas
        # that died are pruned by the actuator, so indices and ports can diverge)
        used = set(self.ports(v))
        port = int(ln.get("portBase", 8200))
        while port in used:
            port += 1
        return self._launch_cmd(v, ln, port)

    def ports(self, v: Variant) -> list[int]:
        """Ports of the variant's live replicas, in start order (read back from
        each process's ``--port`` argument, the single source of truth)."""
        out = []
        for p, _ in self.actuator.procs.get(v.name, []):
            if p.poll() is None and "--port" in p.args:
                out.append(int(p.args[p.args.index("--port") + 1]))
        return out

    def scale(self, v: Variant, n: int):
        n = max(v.min_replicas, min(v.max_replicas, n))
        before = v.current
        if n < before:  # stop routing to the replicas first, then stop them
            self._write_endpoints(exclude={(v.name, p) for p in self.ports(v)[n:]})
        self.actuator.scale(v, n)
        if n != before:
            log.info("variant %s: %d -> %d replicas", v.name, before, v.current)

    # ------------------------------------------------------------ observation
    def _observe(self, v: Variant):
        reps = []
        for port in self.ports(v):
            text = _get(f"http://127.0.0.1:{port}/metrics")
            if text is None:
                reps.append(ReplicaMetrics(pod=f"{v.name}-{port}", ready=False))
                continue
            m = parse_prometheus(text)
            info = (m.get("vllm:cache_config_info") or [({}, 0)])[0][0]
            r = ReplicaMetrics(pod=f"{v.name}-{port}", kv_usage=_first(m, "vllm:kv_cache_usage_perc"),
                               queue_len=_first(m, "vllm:num_requests_waiting"),
                               running=_first(m, "vllm:num_requests_running"),
                               num_gpu_blocks=int(float(info.get("num_gpu_blocks", 0) or 0)),
                               block_size=int(float(info.get("block_size", 16) or 16)))
            reps.append(r)
            if r.queue_len > 0 or r.running > 0:
                self.last_activity[v.model_id] = time.monotonic()
        v.replicas = reps

    def _epp_queue(self) -> dict[str, float]:
        if not self.epp_metrics_url:
            return {}
        text = _get(self.epp_metrics_url)
        if text is None:
            return {}
        out: dict[str, float] = {}
        for labels, val in parse_prometheus(text).get("inference_extension_flow_control_queue_size", []):
            model = labels.get("target_model_name") or labels.get("model_name") or ""
            for m in {v.model_id for v in self.variants.values()}:
                if not model or model == m:
                    out[m] = out.get(m, 0.0) + float(val)
        for m, q in out.items():
            if q > 0:
                self.last_activity[m] = time.monotonic()
        return out

    def pools(self) -> dict[str, list[Variant]]:
        out: dict[str, list[Variant]] = {}
        for v in self.variants.values():
            out.setdefault(v.model_id, []).append(v)
        return out

    # ------------------------------------------------------------ loops
    def reconcile(self) -> dict[str, dict[str, int]]:
        with self.lock:
            for v in self.variants.values():
                self._observe(v)
            q = self._epp_queue()
            now = time.monotonic()
            retained = {m: float(now - self.last_activity.get(m, -1e18) < self.retention) for m in self.pools()}
            decisions = self.engine.step(self.pools(), epp_queue=q, requests_in_retention=retained)
            for m, dec in decisions.items():
                for name, n in dec.items():
                    self.scale(self.variants[name], n)
            self._write_endpoints()
            return decisions

    def fast(self):
        with self.lock:
            q = self._epp_queue()
            before = {n: v.current for n, v in self.variants.items()}
            self.engine.fast_step(self.pools(), q)
            for v in self.variants.values():
                if v.desired != before[v.name] and before[v.name] == 0:
                    self.scale(v, v.desired)

    def start(self):
        for v in self.variants.values():  # start at minReplicas
            self.scale(v, v.min_replicas)
            v.desired = v.current
        self._write_endpoints()

        def loop(fn, period):
            while not self.stop_ev.wait(period):
                try:
                    fn()
                except Exception:  # noqa: BLE001 - keep the controller alive
                    log.exception("wva loop iteration failed")
        self.threads = [threading.Thread(target=loop, args=(self.reconcile, self.interval), daemon=True),
                        threading.Thread(target=loop, args=(self.fast, self.fast_interval), daemon=True)]
        for t in self.threads:
            t.start()
        return self

    def stop(self):
        self.stop_ev.set()
        for t in getattr(self, "threads", []):
            t.join(timeout=5)
        self.actuator.shutdown()

    # ------------------------------------------------------------ outputs
    def _write_endpoints(self, exclude: set = frozenset()):
        if not self.endpoints_file:
            return
        eps = []
        for v in self.variants.values():
            for port in self.ports(v):
                if (v.name, port) in exclude or _get(f"http://127.0.0.1:{port}/health", 0.5) is None:
                    continue
                eps.append({"name": f"{v.name}-{port}", "address": "127.0.0.1", "port": port,
                            "labels": {"llm-d.ai/role": "prefill-decode", "llm-d.ai/model": v.model_id,
                                       "llm-d.ai/variant": v.name}})
        tmp = self.endpoints_file + ".tmp"
        with open(tmp, "w") as f:
            yaml.safe_dump({"endpoints": eps}, f)
        os.replace(tmp, self.endpoints_file)  # atomic: the router's watcher never sees a torn file

    def render_metrics(self) -> str:
        lines = ["# HELP wva_desired_replicas Replica count the optimizer wants for the variant",
                 "# TYPE wva_desired_replicas gauge",
                 "# HELP wva_current_replicas Replicas running for the variant",
                 "# TYPE wva_current_replicas gauge",
                 "# HELP wva_desired_ratio desired / current replicas",
                 "# TYPE wva_desired_ratio gauge"]
        for v in self.variants.values():
            lab = f'variant_name="{v.name}",exported_namespace="{self.namespace}",model_id="{v.model_id}"'
            lines.append(f"wva_desired_replicas{{{lab}}} {v.desired}")
            lines.append(f"wva_current_replicas{{{lab}}} {v.current}")
            lines.append(f"wva_desired_ratio{{{lab}}} {v.desired / v.current if v.current else float(v.desired)}")
        return "\n".join(lines) + "\n"


def main(argv=None):
    from aiohttp import web

    ap = argparse.ArgumentParser("llmd-amd wva controller")
    ap.add_argument("--config", required=True, help="YAML: variantAutoscalings + launch recipes + scalingConfig")
    ap.add_argument("--metrics-bind-address", default=":8080")
    ap.add_argument("--log-level", default="info")
    a = ap.parse_args(argv)
    logging.basicConfig(level=a.log_level.upper(), format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    with open(a.config) as f:
        cfg = yaml.safe_load(f)
    ctl = WVAController(cfg).start()
    app = web.Application()

    async def metrics(_req):
        return web.Response(text=ctl.render_metrics(), content_type="text/plain")

    app.router.add_get("/metrics", metrics)
    host, _, port = a.metrics_bind_address.rpartition(":")
    try:
        web.run_app(app, host=host or "0.0.0.0", port=int(port), access_log=None)
    finally:
        ctl.stop()


if __name__ == "__main__":
    main()
