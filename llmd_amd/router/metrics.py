"""EPP Prometheus metrics: request handling, scheduler, prefix
indexer, flow control, pool gauges. Metric names follow the reference
(docs/architecture/core/router/epp/{request-handling,scheduling,flow-control}.md,
docs/operations/observability/metrics.md:91-122); each family is exported
under the legacy ``inference_*`` names the dashboards/PromQL cookbook use.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

from ..utils.prom import Deferred as _Deferred
from ..utils.prom import Flusher as _Flusher

LAT = (0.005, 0.025, 0.05, 0.1, 0.2, 0.4, 0.6, 0.8, 1.0, 1.25, 1.5, 2, 3, 4, 5, 6, 8, 10, 15, 20, 30, 45,
       60, 120, 180, 240, 300, 360, 480, 600, 900, 1200, 1800, 2700, 3600)
SMALL = (0.0001, 0.0002, 0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1)
SMALL_LAT = tuple(sorted(set(SMALL + (0.25, 0.5, 1, 2, 5, 10, 30, 60, 120, 300, 600))))
TOKS = (1, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32778, 65536, 131072)


class EPPMetrics:
    def __init__(self, pool: str = "pool"):
        self._children: dict = {}
        self._deferred: list[_Deferred] = []
        self.reg = r = CollectorRegistry()
        r.register(_Flusher(self))
        self.pool = pool
        ml = ["model_name", "target_model_name"]
        self.req_total = Counter("inference_objective_request", "Requests", ml + ["priority"], registry=r)
        self.req_err = Counter("inference_objective_request_error", "Errors", ml + ["error_code"], registry=r)
        self.running = Gauge("inference_objective_running_requests", "Running requests", ["model_name"], registry=r)
        self.duration = Histogram("inference_objective_request_duration_seconds", "E2E latency", ml,
                                  buckets=LAT, registry=r)
        self.ttft = Histogram("inference_objective_request_ttft_seconds", "TTFT", ml, buckets=LAT, registry=r)
        self.ntpot = Histogram("inference_objective_normalized_time_per_output_token_seconds", "NTPOT", ml,
                               buckets=SMALL_LAT, registry=r)
        self.pred_ttft = Histogram("inference_objective_request_predicted_ttft_seconds", "Predicted TTFT", ml,
                                   buckets=LAT, registry=r)
        self.pred_tpot = Histogram("inference_objective_request_predicted_tpot_seconds", "Predicted TPOT", ml,
                                   buckets=SMALL_LAT, registry=r)
        self.slo_viol = Counter("inference_objective_request_slo_violation", "SLO violations", ml + ["type"],
                                registry=r)
        self.req_sizes = Histogram("inference_objective_request_sizes", "Request bytes", ml,
                                   buckets=(64, 256, 1024, 4096, 16384, 65536, 262144, 1048576, 4194304), registry=r)
        self.in_toks = Histogram("inference_objective_input_tokens", "Input tokens", ml, buckets=TOKS, registry=r)
        self.out_toks = Histogram("inference_objective_output_tokens", "Output tokens", ml, buckets=TOKS, registry=r)
        self.cached_toks = Histogram("inference_objective_prompt_cached_tokens", "Cached prompt tokens", ml,
                                     buckets=TOKS, registry=r)
        self.rewrite = Counter("inference_extension_model_rewrite_decisions", "Model rewrite decisions",
                               ["model_rewrite_name", "model_name", "target_model"], registry=r)
        # scheduler
        self.sched_attempts = Counter("inference_extension_scheduler_attempts", "Scheduling attempts",
                                      ["status", "target_model_name", "pod_name", "namespace", "port"], registry=r)
        self.sched_e2e = Histogram("inference_extension_scheduler_e2e_duration_seconds", "Scheduling latency",
                                   buckets=SMALL, registry=r)
        self.plugin_dur = Histogram("inference_extension_plugin_duration_seconds", "Plugin latency",
                                    ["extension_point", "plugin_type", "plugin_name"], buckets=SMALL, registry=r)
        self.prefix_size = Gauge("inference_extension_prefix_indexer_size", "Prefix indexer size", registry=r)
        self.prefix_hit = Histogram("inference_extension_prefix_indexer_hit_ratio", "Prefix hit ratio",
                                    buckets=(0, .1, .2, .3, .4, .5, .6, .7, .8, .9, 1.0), registry=r)
        self.pd_decisions = Counter("llm_d_router_epp_pd_decision", "P/D disaggregation decisions",
                                    ["model_name", "decision_type"], registry=r)
        self.info = Gauge("inference_extension_info", "EPP build info", ["commit", "build_ref"], registry=r)
        self.info.labels("llmd-amd", "v0.1").set(1)
        # pool
        self.pool_ready = Gauge("inference_pool_ready_pods", "Ready pods", ["name"], registry=r)
        self.pool_kv = Gauge("inference_pool_average_kv_cache_utilization", "Avg KV util", ["name"], registry=r)
        self.pool_queue = Gauge("inference_pool_average_queue_size", "Avg queue", ["name"], registry=r)
        self.pool_pod_queue = Gauge("inference_pool_per_pod_queue_size", "Per-pod queue",
                                    ["model_server_pod", "name"], registry=r)
        self.pool_running = Gauge("inference_pool_average_running_requests", "Avg running", ["name"], registry=r)
        # flow control
        fl = ["fairness_id", "priority", "inference_pool", "model_name", "target_model_name"]
        self.fc_qsize = Gauge("inference_extension_flow_control_queue_size", "Queued requests", fl, registry=r)
        self.fc_qbytes = Gauge("inference_extension_flow_control_queue_bytes", "Queued bytes", fl, registry=r)
        self.fc_qdur = Histogram("inference_extension_flow_control_request_queue_duration_seconds",
                                 "Time in queue", fl + ["outcome"], buckets=SMALL_LAT, registry=r)
        self.fc_sat = Gauge("inference_extension_flow_control_pool_saturation", "Pool saturation",
                            ["inference_pool"], registry=r)
        self.fc_dispatch = Histogram("inference_extension_flow_control_dispatch_cycle_duration_seconds",
                                     "Dispatch cycle", buckets=SMALL, registry=r)

    # ---------------------------------------------------------------- hooks
    def fc_enqueue(self, req, fc):
        lab = (req.fairness_id, str(req.priority), self.pool, req.model, req.target_model)
        self.fc_qsize.labels(*lab).inc()
        self.fc_qbytes.labels(*lab).inc(max(1, req.raw_size))

    def fc_done(self, req, outcome, waited, fc):
        lab = (req.fairness_id, str(req.priority), self.pool, req.model, req.target_model)
        self.fc_qsize.labels(*lab).dec()
        self.fc_qbytes.labels(*lab).dec(max(1, req.raw_size))
        self.fc_qdur.labels(*lab, outcome).observe(waited)

    def observe_prediction(self, req, pred):
        self.pred_ttft.labels(req.model, req.target_model).observe(pred["ttft_ms"] / 1000.0)
        self.pred_tpot.labels(req.model, req.target_model).observe(pred["tpot_ms"] / 1000.0)

    def pool_update(self, eps, sat: float | None = None):
        from .types import KV_USAGE, RUNNING, WAITING

        n = len(eps)
        self.pool_ready.labels(self.pool).set(n)
        if n:
            self.pool_kv.labels(self.pool).set(sum(float(e.metric(KV_USAGE, 0)) for e in eps) / n)
            self.pool_queue.labels(self.pool).set(sum(float(e.metric(WAITING, 0)) for e in eps) / n)
            self.pool_running.labels(self.pool).set(sum(float(e.metric(RUNNING, 0)) for e in eps) / n)
            for e in eps:
                self.pool_pod_queue.labels(e.name, self.pool).set(float(e.metric(WAITING, 0)))
        if sat is not None:
            self.fc_sat.labels(self.pool).set(sat)

    def child(self, metric, *labels):
        """Cached labelled child: prometheus ``labels()`` costs a few microseconds and
        the request path touches ~15 children per request."""
        key = (id(metric), labels)
        c = self._children.get(key)
        if c is None:
            c = metric.labels(*labels)
            if isinstance(metric, (Counter, Histogram)):
                c = _Deferred(c)
                self._deferred.append(c)
            self._children[key] = c
        return c

    def flush(self):
        for c in list(self._deferred):
            c.flush()

    def render(self) -> bytes:
        return generate_latest(self.reg)
