"""Engine Prometheus metrics with vLLM-compatible names.

The router's ``core-metrics-extractor`` and the reference Grafana dashboards
read these names unchanged (docs/architecture/core/model-servers.md:36-73,
docs/operations/observability/metrics.md:48-72). Each engine owns a private
registry so several engines can live in one process (tests, DP launcher).
Also keeps in-process summaries (TTFT/ITL lists) for the benchmark harness.
"""
from __future__ import annotations

import collections
import time
from typing import Optional

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

from ..utils.prom import Deferred, Flusher

TTFT_BUCKETS = (0.001, 0.005, 0.01, 0.02, 0.04, 0.06, 0.08, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0,
                7.5, 10.0, 20.0, 40.0, 80.0, 160.0, 640.0, 2560.0)
ITL_BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.015, 0.02, 0.025, 0.03, 0.04, 0.05, 0.075, 0.1, 0.15,
               0.2, 0.3, 0.4, 0.5, 0.75, 1.0, 2.5, 5.0, 7.5, 10.0, 20.0, 40.0, 80.0)
REQ_BUCKETS = (0.3, 0.5, 0.8, 1.0, 1.5, 2.0, 2.5, 5.0, 10.0, 15.0, 20.0, 30.0, 40.0, 50.0, 60.0,
               120.0, 240.0, 480.0, 960.0, 1920.0, 7680.0)
TOK_BUCKETS = (1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, 2000, 5000, 10000, 20000, 50000, 100000)


class EngineMetrics:
    def __init__(self, model_name: str, block_size: int, num_gpu_blocks: int,
                 registry: Optional[CollectorRegistry] = None, max_lora: int = 0):
        self.reg = registry or CollectorRegistry()
        self.reg.register(Flusher(self))  # before the families: a scrape sees the batched per-token series
        L = ["model_name"]
        self.model = model_name
        r = self.reg
        self.running = Gauge("vllm:num_requests_running", "Requests in model execution batches", L, registry=r)
        self.waiting = Gauge("vllm:num_requests_waiting", "Requests waiting to be processed", L, registry=r)
        self.kv_usage = Gauge("vllm:kv_cache_usage_perc", "KV-cache usage. 1 means 100 percent usage", L, registry=r)
        self.cache_info = Gauge("vllm:cache_config_info", "Information of the LLMEngine CacheConfig",
                                ["block_size", "num_gpu_blocks", "enable_prefix_caching"], registry=r)
        self.cache_info.labels(str(block_size), str(num_gpu_blocks), "True").set(1)
        self.lora_info = Gauge("vllm:lora_requests_info", "Running stats on lora requests",
                               ["max_lora", "running_lora_adapters", "waiting_lora_adapters"], registry=r)
        self.max_lora = max_lora
        self.prefix_hits = Counter("vllm:prefix_cache_hits", "Prefix cache hits, in tokens", L, registry=r)
        self.prefix_queries = Counter("vllm:prefix_cache_queries", "Prefix cache queries, in tokens", L, registry=r)
        self.prompt_tokens = Counter("vllm:prompt_tokens", "Number of prefill tokens processed", L, registry=r)
        self.gen_tokens = Counter("vllm:generation_tokens", "Number of generation tokens processed", L, registry=r)
        self.preemptions = Counter("vllm:num_preemptions", "Cumulative number of preemptions", L, registry=r)
        self.success = Counter("vllm:request_success", "Count of successfully processed requests",
                               L + ["finished_reason"], registry=r)
        self.ttft = Histogram("vllm:time_to_first_token_seconds", "Time to first token", L,
                              buckets=TTFT_BUCKETS, registry=r)
        self.itl = Histogram("vllm:inter_token_latency_seconds", "Inter-token latency", L,
                             buckets=ITL_BUCKETS, registry=r)
        self.tpot = Histogram("vllm:request_time_per_output_token_seconds", "Time per output token", L,
                              buckets=ITL_BUCKETS, registry=r)
        self.e2e = Histogram("vllm:e2e_request_latency_seconds", "End to end request latency", L,
                             buckets=REQ_BUCKETS, registry=r)
        self.queue_t = Histogram("vllm:request_queue_time_seconds", "Time spent waiting", L,
                                 buckets=REQ_BUCKETS, registry=r)
        self.prefill_t = Histogram("vllm:request_prefill_time_seconds", "Time in prefill", L,
                                   buckets=REQ_BUCKETS, registry=r)
        self.decode_t = Histogram("vllm:request_decode_time_seconds", "Time in decode", L,
                                  buckets=REQ_BUCKETS, registry=r)
        self.req_prompt = Histogram("vllm:request_prompt_tokens", "Prompt tokens per request", L,
                                    buckets=TOK_BUCKETS, registry=r)
        self.req_gen = Histogram("vllm:request_generation_tokens", "Generation tokens per request", L,
                                 buckets=TOK_BUCKETS, registry=r)
        self.iter_tokens = Histogram("vllm:iteration_tokens_total", "Tokens per engine step", L,
                                     buckets=TOK_BUCKETS, registry=r)
        self._last_prefix = (0, 0)
        self._last_preempt = 0
        # in-process summaries for benchmarks (bounded: a long-running server must not grow them forever)
        self.ttfts: collections.deque = collections.deque(maxlen=1 << 16)
        self.itls: collections.deque = collections.deque(maxlen=1 << 16)
        self.n_gen = 0
        self.n_prompt = 0
        self._last_tok_time: dict[str, float] = {}
        self.running.labels(model_name).set(0)
        self.waiting.labels(model_name).set(0)
        self.kv_usage.labels(model_name).set(0)
        # label children of the per-step / per-token series, resolved once (labels() locks and
        # hashes on every call; on_step touches every running request each step)
        # per-token series batched (utils/prom.py Deferred): on_step runs between decode graph
        # replays, one ITL observation per running request
        self._c_itl = Deferred(self.itl.labels(model_name))
        self._c_ttft = Deferred(self.ttft.labels(model_name))
        self._c_iter = self.iter_tokens.labels(model_name)
        self._c_gen = self.gen_tokens.labels(model_name)
        self._deferred = (self._c_itl, self._c_ttft)
        self._c_running = self.running.labels(model_name)
        self._c_waiting = self.waiting.labels(model_name)
        self._c_kv = self.kv_usage.labels(model_name)

    def flush(self):
        for c in self._deferred:
            c.flush()

    def on_arrival(self, r):
        pass

    def on_step(self, so, touched, dt, n_running, n_waiting, usage, prefix_stats):
        m = self.model
        self._c_running.set(n_running)
        self._c_waiting.set(n_waiting)
        self._c_kv.set(usage)
        hits, queries = prefix_stats
        dh, dq = hits - self._last_prefix[0], queries - self._last_prefix[1]
        if dh > 0:
            self.prefix_hits.labels(m).inc(dh)
        if dq > 0:
            self.prefix_queries.labels(m).inc(dq)
        self._last_prefix = (hits, queries)
        if so.preempted:
            self.preemptions.labels(m).inc(len(so.preempted))
        ptoks = sum(s.num_new_tokens for s in so.prefills)
        if ptoks:
            self.prompt_tokens.labels(m).inc(ptoks)
            self.n_prompt += ptoks
        self._c_iter.observe(so.num_tokens)
        ng = len(touched)
        if ng:
            self._c_gen.inc(ng)
            self.n_gen += ng
        now = time.monotonic()
        itl, last_tok = self._c_itl, self._last_tok_time
        for r in touched:
            if len(r.output_token_ids) == 1 and r.first_token_time is not None:
                t = r.first_token_time - r.arrival_time
                self._c_ttft.observe(t)
                self.ttfts.append(t)
            else:
                last = last_tok.get(r.request_id)
                if last is not None:
                    itl.observe(now - last)
                    self.itls.append(now - last)
            last_tok[r.request_id] = now

    def on_finish(self, r):
        m = self.model
        self._last_tok_time.pop(r.request_id, None)
        reason = r.finish_reason or "abort"
        self.success.labels(m, reason).inc()
        if r.finished_time is None:
            return
        self.e2e.labels(m).observe(r.finished_time - r.arrival_time)
        if r.first_scheduled_time is not None:
            self.queue_t.labels(m).observe(r.first_scheduled_time - r.arrival_time)
            if r.first_token_time is not None:
                self.prefill_t.labels(m).observe(r.first_token_time - r.first_scheduled_time)
                self.decode_t.labels(m).observe(r.finished_time - r.first_token_time)
        n = len(r.output_token_ids)
        self.req_prompt.labels(m).observe(r.num_prompt_tokens)
        self.req_gen.labels(m).observe(n)
        if n > 1 and r.first_token_time is not None:
            self.tpot.labels(m).observe((r.finished_time - r.first_token_time) / (n - 1))

    def set_lora(self, running: list[str], waiting: list[str]):
        self.lora_info.clear()
        self.lora_info.labels(str(self.max_lora), ",".join(running), ",".join(waiting)).set(time.time())

    def render(self) -> bytes:
        return generate_latest(self.reg)
