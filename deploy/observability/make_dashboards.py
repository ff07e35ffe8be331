"""Generate the Grafana dashboards (vLLM engine, router/EPP,
P/D transfer, failure & saturation) from panel specs; the metric names are the
ones our engine, router and kvx export (vllm:*, inference_*, vllm:nixl_*).
    python deploy/observability/make_dashboards.py"""
import json
import os

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "grafana", "dashboards")

DASHBOARDS = {
    "llmd-engine": ("llm-d AMD / engine (vLLM metrics)", [
        ("Running / waiting requests", ["sum by (pod) (vllm:num_requests_running)",
                                        "sum by (pod) (vllm:num_requests_waiting)"], "short"),
        ("KV cache usage", ["max by (pod) (vllm:kv_cache_usage_perc)"], "percentunit"),
        ("Output tokens/s", ["sum by (pod) (rate(vllm:generation_tokens_total[1m]))"], "short"),
        ("Prompt tokens/s", ["sum by (pod) (rate(vllm:prompt_tokens_total[1m]))"], "short"),
        ("TTFT p50 / p99", ["histogram_quantile(0.5, sum by (le) (rate(vllm:time_to_first_token_seconds_bucket[5m])))",
                            "histogram_quantile(0.99, sum by (le) (rate(vllm:time_to_first_token_seconds_bucket[5m])))"],
         "s"),
        ("ITL p50 / p99", ["histogram_quantile(0.5, sum by (le) (rate(vllm:inter_token_latency_seconds_bucket[5m])))",
                           "histogram_quantile(0.99, sum by (le) (rate(vllm:inter_token_latency_seconds_bucket[5m])))"],
         "s"),
        ("Prefix cache hit rate", ["sum(rate(vllm:prefix_cache_hits_total[5m])) / "
                                   "sum(rate(vllm:prefix_cache_queries_total[5m]))"], "percentunit"),
        ("Preemptions/s", ["sum by (pod) (rate(vllm:num_preemptions_total[5m]))"], "short"),
        ("Queue time p90", ["histogram_quantile(0.9, sum by (le) (rate(vllm:request_queue_time_seconds_bucket[5m])))"],
         "s"),
        ("Tokens per engine step", ["histogram_quantile(0.5, sum by (le) (rate(vllm:iteration_tokens_total_bucket[5m])))"],
         "short"),
    ]),
    "llmd-router": ("llm-d AMD / router (EPP)", [
        ("Requests/s by model", ["sum by (model_name) (rate(inference_objective_request_total[1m]))"], "reqps"),
        ("Errors/s", ["sum by (error_code) (rate(inference_objective_request_error_total[1m]))"], "reqps"),
        ("E2E latency p90", ["histogram_quantile(0.9, sum by (le) (rate(inference_objective_request_duration_seconds_bucket[5m])))"],
         "s"),
        ("Scheduler attempts", ["sum by (status) (rate(inference_extension_scheduler_attempts_total[1m]))"], "ops"),
        ("Flow-control queue size", ["sum by (priority) (inference_extension_flow_control_queue_size)"], "short"),
        ("Pool saturation", ["max(inference_extension_flow_control_pool_saturation)"], "percentunit"),
        ("Prefix indexer hit ratio", ["avg(inference_extension_prefix_indexer_hit_ratio)"], "percentunit"),
        ("Pool KV utilisation / queue", ["inference_pool_average_kv_cache_utilization",
                                         "inference_pool_average_queue_size"], "short"),
        ("Ready pods", ["inference_pool_ready_pods"], "short"),
        ("P/D decisions", ["sum by (decision_type) (rate(llm_d_router_epp_pd_decision_total[5m]))"], "ops"),
    ]),
    "llmd-pd": ("llm-d AMD / P-D disaggregation (kvx)", [
        ("KV transfer time p50 / p99", ["histogram_quantile(0.5, sum by (le) (rate(vllm:nixl_xfer_time_seconds_bucket[5m])))",
                                        "histogram_quantile(0.99, sum by (le) (rate(vllm:nixl_xfer_time_seconds_bucket[5m])))"],
         "s"),
        ("KV bytes/s pulled", ["sum by (pod) (rate(vllm:nixl_bytes_transferred_sum[1m]))"], "Bps"),
        ("Failed transfers/s", ["sum by (pod) (rate(vllm:nixl_num_failed_transfers_total[5m]))"], "ops"),
        ("Prefill vs decode TTFT", ["histogram_quantile(0.5, sum by (le, pod) (rate(vllm:time_to_first_token_seconds_bucket[5m])))"],
         "s"),
        ("Decode batch (running)", ["sum by (pod) (vllm:num_requests_running)"], "short"),
    ]),
    "llmd-saturation": ("llm-d AMD / failure & saturation", [
        ("KV usage > 80 % (pods)", ["count(vllm:kv_cache_usage_perc > 0.8)"], "short"),
        ("Waiting > 5 (pods)", ["count(vllm:num_requests_waiting > 5)"], "short"),
        ("429 / 503 rejections", ["sum by (error_code) (rate(inference_objective_request_error_total{error_code=~\"429|503\"}[1m]))"],
         "reqps"),
        ("Request success rate", ["sum(rate(vllm:request_success_total[5m]))"], "reqps"),
        ("SLO violations", ["sum(rate(inference_objective_request_slo_violation_total[5m]))"], "ops"),
    ]),
    # KV-cache performance (reference guides/recipes/observability/grafana/dashboards/
    # llm-d-performance-kv-cache.json): latency vs cache hit rate, per pod, plus the offload tiers
    "llmd-kv-cache": ("llm-d AMD / KV-cache performance", [
        ("Time to first token p50 / p90", [
            "histogram_quantile(0.5, sum by (le) (rate(vllm:time_to_first_token_seconds_bucket[5m])))",
            "histogram_quantile(0.9, sum by (le) (rate(vllm:time_to_first_token_seconds_bucket[5m])))"], "s"),
        ("Inter-token latency p50 / p90", [
            "histogram_quantile(0.5, sum by (le) (rate(vllm:inter_token_latency_seconds_bucket[5m])))",
            "histogram_quantile(0.9, sum by (le) (rate(vllm:inter_token_latency_seconds_bucket[5m])))"], "s"),
        ("KV cache hit rate (pool)", ["sum(rate(vllm:prefix_cache_hits_total[5m])) / "
                                      "clamp_min(sum(rate(vllm:prefix_cache_queries_total[5m])), 1)"], "percentunit"),
        ("Per-pod cache hit rate", ["sum by (pod) (rate(vllm:prefix_cache_hits_total[5m])) / "
                                    "clamp_min(sum by (pod) (rate(vllm:prefix_cache_queries_total[5m])), 1)"],
         "percentunit"),
        ("KV cache usage (pool max / mean)", ["max(vllm:kv_cache_usage_perc)", "avg(vllm:kv_cache_usage_perc)"],
         "percentunit"),
        ("Per-pod KV cache usage", ["max by (pod) (vllm:kv_cache_usage_perc)"], "percentunit"),
        ("Request throughput", ["sum(rate(vllm:request_success_total[1m]))"], "reqps"),
        ("Request queue (running / waiting)", ["sum(vllm:num_requests_running)", "sum(vllm:num_requests_waiting)"],
         "short"),
        ("EPP pool health & load", ["inference_pool_ready_pods", "inference_pool_average_queue_size"], "short"),
        ("EPP pool KV utilisation", ["inference_pool_average_kv_cache_utilization"], "percentunit"),
        ("Offload tier traffic (bytes/s)", ["sum by (transfer_type) (rate(vllm:kv_offload_total_bytes[1m]))"], "Bps"),
        ("Offload transfer size p50", ["histogram_quantile(0.5, sum by (le, transfer_type) "
                                       "(rate(vllm:kv_offload_size_bucket[5m])))"], "bytes"),
        ("Host-tier occupancy", ["max by (pod) (vllm:kv_offload_cpu_usage_perc)"], "percentunit"),
    ]),
    # Diagnostic drill-down (reference llm-d-diagnostic-drilldown-dashboard.json): serving,
    # routing, prefix caching and P/D sections
    "llmd-drilldown": ("llm-d AMD / diagnostic drill-down", [
        ("Model serving: running per pod", ["sum by (pod) (vllm:num_requests_running)"], "short"),
        ("KV cache utilisation per pod", ["max by (pod) (vllm:kv_cache_usage_perc)"], "percentunit"),
        ("Request queue lengths", ["sum by (pod) (vllm:num_requests_waiting)"], "short"),
        ("Model throughput (req/s)", ["sum by (pod) (rate(vllm:request_success_total[1m]))"], "reqps"),
        ("Generation token rate", ["sum by (pod) (rate(vllm:generation_tokens_total[1m]))"], "short"),
        ("Queue utilisation (waiting / max-num-seqs)", [
            "sum by (pod) (vllm:num_requests_waiting) / clamp_min(sum by (pod) (vllm:num_requests_running), 1)"],
         "percentunit"),
        ("Routing: request distribution", ["sum by (pod) (rate(vllm:prompt_tokens_total[1m])) / "
                                           "clamp_min(sum(rate(vllm:prompt_tokens_total[1m])), 1)"], "percentunit"),
        ("Token distribution (prompt tok/s by pod)", ["sum by (pod) (rate(vllm:prompt_tokens_total[1m]))"], "short"),
        ("Idle GPU time (pods with no running requests)", ["count(sum by (pod) (vllm:num_requests_running) == 0)"],
         "short"),
        ("Routing decision latency p50 / p99", [
            "histogram_quantile(0.5, sum by (le) (rate(inference_extension_scheduler_e2e_duration_seconds_bucket[5m])))",
            "histogram_quantile(0.99, sum by (le) (rate(inference_extension_scheduler_e2e_duration_seconds_bucket[5m])))"],
         "s"),
        ("Prefix cache hit rate", ["sum(rate(vllm:prefix_cache_hits_total[5m])) / "
                                   "clamp_min(sum(rate(vllm:prefix_cache_queries_total[5m])), 1)"], "percentunit"),
        ("Per-instance hit rate", ["sum by (pod) (rate(vllm:prefix_cache_hits_total[5m])) / "
                                   "clamp_min(sum by (pod) (rate(vllm:prefix_cache_queries_total[5m])), 1)"],
         "percentunit"),
        ("P/D: prefill worker utilisation", ["avg(vllm:num_requests_running{llm_d_ai_role=\"prefill\"})"], "short"),
        ("P/D: decode worker utilisation", ["avg(vllm:kv_cache_usage_perc{llm_d_ai_role=\"decode\"})"],
         "percentunit"),
        ("P/D: prefill queue length", ["sum(vllm:num_requests_waiting{llm_d_ai_role=\"prefill\"})"], "short"),
        ("P/D decisions", ["sum by (decision_type) (rate(llm_d_router_epp_pd_decision_total[5m]))"], "ops"),
    ]),
}


def panel(i, title, exprs, unit):
    return {"id": i + 1, "type": "timeseries", "title": title,
            "gridPos": {"h": 8, "w": 12, "x": 12 * (i % 2), "y": 8 * (i // 2)},
            "datasource": {"type": "prometheus", "uid": "${datasource}"},
            "fieldConfig": {"defaults": {"unit": unit}, "overrides": []},
            "targets": [{"refId": chr(65 + j), "expr": e, "legendFormat": "__auto"} for j, e in enumerate(exprs)]}


def dashboard(uid, title, panels):
    return {"uid": uid, "title": title, "schemaVersion": 39, "version": 1, "refresh": "10s",
            "time": {"from": "now-1h", "to": "now"}, "tags": ["llm-d", "mi355x"],
            "templating": {"list": [{"name": "datasource", "type": "datasource", "query": "prometheus"}]},
            "panels": [panel(i, *p) for i, p in enumerate(panels)]}


def main():
    os.makedirs(HERE, exist_ok=True)
    for uid, (title, panels) in DASHBOARDS.items():
        with open(os.path.join(HERE, uid + ".json"), "w") as f:
            json.dump(dashboard(uid, title, panels), f, indent=1)


if __name__ == "__main__":
    main()
