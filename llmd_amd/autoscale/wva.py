"""Workload Variant Autoscaler (reference
docs/architecture/advanced/autoscaling/wva.md:1-401) and the HPA/KEDA signal
mapping (C32, docs/architecture/advanced/autoscaling/hpa-keda.md:30-95).

Pipeline per InferencePool (= model id): Analyzer -> Optimizer -> Enforcer.

Analyzers
* ``PercentageSaturationAnalyzer`` (default): a replica is saturated when KV
  usage >= kvCacheThreshold (0.80) or queue >= queueLengthThreshold (5);
  scale-up when average spare KV < kvSpareTrigger (0.10) or spare queue <
  queueSpareTrigger (3); scale-down when >= 2 non-saturated replicas exist and
  an N/(N-1) redistribution keeps both spares above their triggers. All
  scaling is blocked while any variant is transitioning.
* ``TokenSaturationAnalyzer``: per-replica capacity = min(k1, k2) tokens with
  k1 = KV tokens x threshold and k2 from the priority chain observed (queue
  saturated) -> history (window 10, bucketed by output length) -> derived
  from max-num-batched-tokens / max-num-seqs -> k1. Demand = tokens in use +
  queue x avg input (+ EPP queue); required = demand / 0.85 - supply, spare
  = supply - demand / 0.70.
* ``SLOAnalyzer``: a linear Kalman filter learns (alpha, beta, gamma) of the
  iteration-time model ``t(n) = alpha + beta*n + gamma*n*ctx`` from observed
  TTFT / ITL; a state-dependent M/M/1/K model (service rate of n in system =
  n / (osl * t(n))) gives the max arrival rate per replica that meets the
  TTFT / ITL targets (explicit, or idle latency x sloMultiplier 3.0).
Optimizers: cost-aware (scale up the cheapest variant, down the most
expensive) and greedy-by-score (fair-share a GPU budget by priority).
Enforcer: scale-to-zero after a retention period without requests (10 min)
or keep >= 1 replica on the cheapest variant; ``ScaleFromZero`` polls the EPP
flow-control queue and wakes idle pools.

Single-node actuation (``ProcessActuator``): a variant is an engine launch
recipe with a GPU count; replicas are engine processes started on free GPUs
(``HIP_VISIBLE_DEVICES``) and stopped in reverse order.
"""
from __future__ import annotations

import math
import os
import signal
import subprocess
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np


# ------------------------------------------------------------------ model
@dataclass
class ReplicaMetrics:
    pod: str
    kv_usage: float = 0.0                 # vllm:kv_cache_usage_perc
    queue_len: float = 0.0                # vllm:num_requests_waiting
    running: float = 0.0                  # vllm:num_requests_running
    num_gpu_blocks: int = 0               # vllm:cache_config_info
    block_size: int = 16
    avg_input_tokens: float = 0.0
    avg_output_tokens: float = 0.0
    max_num_batched_tokens: int = 8192
    max_num_seqs: int = 256
    ready: bool = True
    arrival_rate: float = 0.0             # scheduler attempts success rate (req/s)
    avg_ttft: float = 0.0                 # seconds
    avg_itl: float = 0.0                  # seconds

    @property
    def kv_tokens(self) -> int:
        return self.num_gpu_blocks * self.block_size

    @property
    def tokens_in_use(self) -> float:
        return self.kv_usage * self.kv_tokens


@dataclass
class Variant:
    """A VariantAutoscaling object (spec + status)."""
    name: str
    model_id: str
    min_replicas: int = 1
    max_replicas: int = 2
    cost: float = 10.0
    gpus_per_replica: int = 1
    current: int = 0
    desired: int = 0
    replicas: list[ReplicaMetrics] = field(default_factory=list)

    @property
    def transitioning(self) -> bool:
        return self.desired != self.current


@dataclass
class ScalingRequest:
    model_id: str
    required: float = 0.0      # >0: capacity (replicas or tokens) to add
    spare: float = 0.0         # >0: capacity that can be removed
    priority: float = 1.0
    unit: str = "replicas"     # or "tokens"
    desired_replicas: Optional[int] = None  # SLO analyzer: absolute target


# --------------------------------------------------------------- analyzers
class PercentageSaturationAnalyzer:
    def __init__(self, kvCacheThreshold=0.80, queueLengthThreshold=5, kvSpareTrigger=0.10,
                 queueSpareTrigger=3, **_):
        self.kv_t, self.q_t = kvCacheThreshold, queueLengthThreshold
        self.kv_spare, self.q_spare = kvSpareTrigger, queueSpareTrigger

    def analyze(self, model_id: str, variants: list[Variant], epp_queue: float = 0.0) -> ScalingRequest:
        req = ScalingRequest(model_id)
        if any(v.transitioning for v in variants):
            return req
        reps = [r for v in variants for r in v.replicas if r.ready]
        if not reps:
            req.required = 1.0 if epp_queue > 0 else 0.0
            return req
        kv_sp = float(np.mean([max(0.0, self.kv_t - r.kv_usage) for r in reps]))
        q_sp = float(np.mean([max(0.0, self.q_t - r.queue_len) for r in reps]))
        if kv_sp < self.kv_spare or q_sp < self.q_spare:
            req.required = 1.0
            return req
        ok = [r for r in reps if r.kv_usage < self.kv_t and r.queue_len < self.q_t]
        n = len(reps)
        if len(ok) >= 2 and n >= 2:
            f = n / (n - 1)
            kv2 = float(np.mean([max(0.0, self.kv_t - r.kv_usage * f) for r in reps]))
            q2 = float(np.mean([max(0.0, self.q_t - r.queue_len * f) for r in reps]))
            if kv2 >= self.kv_spare and q2 >= self.q_spare:
                req.spare = 1.0
        return req


class TokenSaturationAnalyzer:
    HISTORY = 10

    def __init__(self, kvCacheThreshold=0.80, queueLengthThreshold=5, scaleUpThreshold=0.85,
                 scaleDownBoundary=0.70, **_):
        self.kv_t, self.q_t = kvCacheThreshold, queueLengthThreshold
        self.up, self.down = scaleUpThreshold, scaleDownBoundary
        self.k2_hist: dict[tuple[str, str], deque] = {}
        self.capacity_cache: dict[str, float] = {}  # variant -> per-replica capacity (for zero replicas)

    @staticmethod
    def _bucket(osl: float) -> str:
        return "short" if osl < 100 else ("medium" if osl < 500 else "long")

    def k2(self, v: Variant, r: ReplicaMetrics) -> float:
        key = (v.name, self._bucket(r.avg_output_tokens))
        h = self.k2_hist.setdefault(key, deque(maxlen=self.HISTORY))
        if r.queue_len >= self.q_t and r.tokens_in_use > 0:   # observed: compute-saturated now
            h.append(r.tokens_in_use)
            return r.tokens_in_use
        if h:                                                 # historical
            return float(np.mean(h))
        if r.avg_input_tokens > 0 and r.avg_output_tokens > 0:  # derived steady-state batching model
            isl, osl = r.avg_input_tokens, r.avg_output_tokens
            # concurrent sequences limited by max_num_seqs and by the chunked-prefill
            # token budget: each step admits (mnbt - n) prefill tokens -> n <= mnbt*osl/(isl+osl)
            n = min(r.max_num_seqs, r.max_num_batched_tokens * osl / (isl + osl))
            return n * (isl + osl / 2)
        return r.kv_tokens * self.kv_t                        # fallback: memory-only

    def capacity(self, v: Variant, r: ReplicaMetrics) -> float:
        return min(r.kv_tokens * self.kv_t, self.k2(v, r))

    def analyze(self, model_id: str, variants: list[Variant], epp_queue: float = 0.0,
                epp_queue_tokens: float = 0.0) -> ScalingRequest:
        req = ScalingRequest(model_id, unit="tokens")
        supply = demand = anticipated = 0.0
        avg_in = []
        for v in variants:
            ready = [r for r in v.replicas if r.ready]
            caps = [self.capacity(v, r) for r in ready]
            if caps:
                self.capacity_cache[v.name] = float(np.median(caps))
            per = self.capacity_cache.get(v.name, 0.0)
            supply += per * len(ready)
            anticipated += per * max(0, v.desired - len(ready))  # pending replicas
            for r in ready:
                demand += r.tokens_in_use + r.queue_len * r.avg_input_tokens
                avg_in.append(r.avg_input_tokens)
        demand += epp_queue_tokens or epp_queue * (float(np.mean(avg_in)) if avg_in else 0.0)
        req.required = max(0.0, demand / self.up - supply - anticipated)
        req.spare = max(0.0, supply - demand / self.down)
        return req


class KalmanTuner:
    """Linear Kalman filter on theta = (alpha, beta, gamma) [seconds].

    Observations per snapshot (n = concurrency, isl, osl):
      ITL  = alpha + beta*n + gamma*n*(isl + osl/2)
      TTFT_service = alpha + beta*isl        (prefill of one request)
    """

    def __init__(self, theta0=(0.005, 1e-4, 1e-8), p0=1.0, q=1e-6, r=1e-4):
        self.x = np.array(theta0, dtype=np.float64)
        self.P = np.diag([p0 * 1e-4, p0 * 1e-8, p0 * 1e-14])
        self.Q = np.diag([q * 1e-4, q * 1e-8, q * 1e-14])
        self.R = np.eye(2) * r
        self.n_updates = 0

    def update(self, n: float, isl: float, osl: float, ttft_service: float, itl: float):
        H = np.array([[1.0, n, n * (isl + osl / 2)], [1.0, isl, 0.0]])
        z = np.array([itl, ttft_service])
        P = self.P + self.Q
        S = H @ P @ H.T + self.R * max(1e-12, float(z @ z))
        K = P @ H.T @ np.linalg.inv(S)
        self.x = self.x + K @ (z - H @ self.x)
        self.x = np.maximum(self.x, 0.0)
        self.P = (np.eye(3) - K @ H) @ P
        self.n_updates += 1

    def iter_time(self, n: float, ctx: float) -> float:
        a, b, g = self.x
        return a + b * n + g * n * ctx

    def prefill_time(self, isl: float) -> float:
        a, b, _ = self.x
        return a + b * isl


def mm1k_latency(lam: float, tuner: KalmanTuner, isl: float, osl: float, K: int) -> tuple[float, float, float]:
    """State-dependent M/M/1/K with batch service: returns (ttft, itl, loss)."""
    ctx = isl + osl / 2
    p = [1.0]
    for n in range(1, K + 1):
        mu = n / max(1e-9, osl * tuner.iter_time(n, ctx) + tuner.prefill_time(isl))
        p.append(p[-1] * lam / mu)
        if p[-1] > 1e300:
            break
    p = np.array(p)
    p /= p.sum()
    ns = np.arange(len(p))
    L = float((ns * p).sum())
    loss = float(p[-1])
    thr = lam * (1 - loss)
    W = L / max(thr, 1e-12)  # Little: time in system
    service = osl * float((p[1:] * [tuner.iter_time(n, ctx) for n in ns[1:]]).sum() / max(1e-12, p[1:].sum())) \
        if len(p) > 1 else osl * tuner.iter_time(1, ctx)
    itl = service / max(1.0, osl)
    ttft = max(0.0, W - service) + tuner.prefill_time(isl)
    return ttft, itl, loss


class SLOAnalyzer:
    def __init__(self, sloMultiplier: float = 3.0, targetTTFT: Optional[float] = None,
                 targetITL: Optional[float] = None, tuningEnabled: bool = True, max_batch: int = 256, **_):
        self.k = sloMultiplier
        self.t_ttft = targetTTFT / 1000 if targetTTFT else None
        self.t_itl = targetITL / 1000 if targetITL else None
        self.tuning = tuningEnabled
        self.K = max_batch
        self.tuner = KalmanTuner()

    def observe(self, r: ReplicaMetrics):
        if self.tuning and r.avg_itl > 0 and r.avg_ttft > 0 and r.avg_input_tokens > 0:
            self.tuner.update(max(1.0, r.running), r.avg_input_tokens, max(1.0, r.avg_output_tokens),
                              r.avg_ttft, r.avg_itl)

    def targets(self, isl: float, osl: float) -> tuple[float, float]:
        ttft = self.t_ttft or self.k * self.tuner.prefill_time(isl)
        itl = self.t_itl or self.k * self.tuner.iter_time(1, isl + osl / 2)
        return ttft, itl

    def max_rate(self, isl: float, osl: float) -> float:
        t_ttft, t_itl = self.targets(isl, osl)
        lo, hi = 0.0, 1.0
        while hi < 1e6:
            ttft, itl, loss = mm1k_latency(hi, self.tuner, isl, osl, self.K)
            if ttft > t_ttft or itl > t_itl or loss > 0.01:
                break
            lo, hi = hi, hi * 2
        for _ in range(40):
            mid = (lo + hi) / 2
            ttft, itl, loss = mm1k_latency(mid, self.tuner, isl, osl, self.K)
            if ttft <= t_ttft and itl <= t_itl and loss <= 0.01:
                lo = mid
            else:
                hi = mid
        return lo

    def analyze(self, model_id: str, variants: list[Variant], **_) -> ScalingRequest:
        reps = [r for v in variants for r in v.replicas if r.ready]
        for r in reps:
            self.observe(r)
        lam = sum(r.arrival_rate for r in reps)
        isl = float(np.mean([r.avg_input_tokens for r in reps])) if reps else 0.0
        osl = float(np.mean([r.avg_output_tokens for r in reps])) if reps else 0.0
        req = ScalingRequest(model_id)
        if lam <= 0 or isl <= 0 or osl <= 0:
            return req
        mr = self.max_rate(isl, osl)
        req.desired_replicas = max(1, math.ceil(lam / mr)) if mr > 0 else None
        return req


# --------------------------------------------------------------- optimizers
class CostAwareOptimizer:
    """Per pool: scale up the cheapest variant with headroom, down the most expensive."""

    def optimize(self, req: ScalingRequest, variants: list[Variant], per_replica_tokens=None) -> dict[str, int]:
        out = {v.name: v.current for v in variants}
        if req.desired_replicas is not None:
            delta = req.desired_replicas - sum(v.current for v in variants)
        elif req.required > 0:
            if req.unit == "tokens":
                v0 = min((v for v in variants if v.current < v.max_replicas), key=lambda v: v.cost, default=None)
                per = (per_replica_tokens or {}).get(v0.name, 0) if v0 else 0
                delta = max(1, math.ceil(req.required / per)) if per > 0 else 1
            else:
                delta = int(math.ceil(req.required))
        elif req.spare > 0:
            if req.unit == "tokens":
                v0 = max((v for v in variants if v.current > v.min_replicas), key=lambda v: v.cost, default=None)
                per = (per_replica_tokens or {}).get(v0.name, 0) if v0 else 0
                delta = -int(req.spare // per) if per > 0 else 0
            else:
                delta = -int(req.spare)
        else:
            delta = 0
        while delta > 0:
            cand = [v for v in variants if out[v.name] < v.max_replicas]
            if not cand:
                break
            v = min(cand, key=lambda v: v.cost)
            out[v.name] += 1
            delta -= 1
        while delta < 0:
            cand = [v for v in variants if out[v.name] > v.min_replicas]
            if not cand:
                break
            v = max(cand, key=lambda v: v.cost)
            out[v.name] -= 1
            delta += 1
        return out


class GreedyByScoreOptimizer:
    """Limited mode: fair-share a GPU budget across pools by priority score."""

    def __init__(self, gpu_budget: int):
        self.budget = gpu_budget

    def optimize_all(self, pools: dict[str, tuple[ScalingRequest, list[Variant]]]) -> dict[str, dict[str, int]]:
        base = CostAwareOptimizer()
        wants = {m: base.optimize(req, vs) for m, (req, vs) in pools.items()}
        alloc = {m: {v.name: min(v.current, wants[m][v.name]) for v in vs} for m, (_, vs) in pools.items()}
        used = sum(alloc[m][v.name] * v.gpus_per_replica for m, (_, vs) in pools.items() for v in vs)
        # grant increments one replica at a time to the pool with the best score
        # (priority x unmet fraction) until the GPU budget runs out
        while True:
            best, best_score = None, 0.0
            for m, (req, vs) in pools.items():
                for v in sorted(vs, key=lambda v: v.cost):
                    if alloc[m][v.name] < wants[m][v.name] and used + v.gpus_per_replica <= self.budget:
                        unmet = (wants[m][v.name] - alloc[m][v.name]) / max(1, wants[m][v.name])
                        s = req.priority * unmet
                        if s > best_score:
                            best, best_score = (m, v), s
                        break
            if best is None:
                break
            m, v = best
            alloc[m][v.name] += 1
            used += v.gpus_per_replica
        return alloc


# ---------------------------------------------------------------- enforcer
class Enforcer:
    def __init__(self, enable_scale_to_zero: bool = False, retention_period_s: float = 600.0):
        self.stz = enable_scale_to_zero
        self.retention = retention_period_s

    def enforce(self, decision: dict[str, int], variants: list[Variant], requests_in_retention: float):
        if self.stz and not any(v.min_replicas > 0 for v in variants) and requests_in_retention == 0:
            return {k: 0 for k in decision}
        if not self.stz and sum(decision.values()) == 0 and variants:
            cheapest = min(variants, key=lambda v: v.cost)
            decision = dict(decision)
            decision[cheapest.name] = max(1, cheapest.min_replicas)
        return decision


class ScaleFromZero:
    """Fast path (100 ms poll): a pool with no replicas and a non-empty EPP
    flow-control queue is scaled to 1 on its cheapest variant."""

    def check(self, variants: list[Variant], epp_queue_size: float) -> Optional[dict[str, int]]:
        if sum(v.current for v in variants) == 0 and epp_queue_size > 0 and variants:
            cheapest = min(variants, key=lambda v: v.cost)
            return {v.name: (1 if v is cheapest else 0) for v in variants}
        return None


# ---------------------------------------------------------------- engine
class WVAEngine:
    """Runs the pipeline over all pools once per interval (default 30 s)."""

    def __init__(self, config: Optional[dict] = None, actuator=None, gpu_budget: Optional[int] = None,
                 elector=None):
        cfg = dict(config or {})
        self.cfg = cfg
        # HA (--leader-elect, wva.md:397-400): only the lease holder analyses and
        # actuates; standbys keep nothing that a takeover would need
        self.elector = elector
        name = cfg.get("analyzerName", "")
        if cfg.get("sloMultiplier") is not None or cfg.get("targetTTFT") is not None:
            self.analyzer = SLOAnalyzer(**cfg)
        elif name == "saturation":
            self.analyzer = TokenSaturationAnalyzer(**cfg)
        else:
            self.analyzer = PercentageSaturationAnalyzer(**cfg)
        self.limited = bool(cfg.get("enableLimiter", False))
        self.optimizer = GreedyByScoreOptimizer(gpu_budget or 8) if self.limited else CostAwareOptimizer()
        self.enforcer = Enforcer(bool(cfg.get("enable_scale_to_zero", False)),
                                 _dur(cfg.get("retention_period", "10m")))
        self.sfz = ScaleFromZero()
        self.actuator = actuator
        self.last_decisions: dict[str, dict[str, int]] = {}

    def step(self, pools: dict[str, list[Variant]], epp_queue: Optional[dict[str, float]] = None,
             requests_in_retention: Optional[dict[str, float]] = None) -> dict[str, dict[str, int]]:
        if self.elector is not None and not self.elector.is_leader:
            return {}
        epp_queue = epp_queue or {}
        reqs = {}
        for m, vs in pools.items():
            reqs[m] = self.analyzer.analyze(m, vs, epp_queue=epp_queue.get(m, 0.0))
            reqs[m].priority = float(self.cfg.get("priority", 1.0))
        if self.limited:
            decisions = self.optimizer.optimize_all({m: (reqs[m], vs) for m, vs in pools.items()})
        else:
            per = getattr(self.analyzer, "capacity_cache", None)
            decisions = {m: self.optimizer.optimize(reqs[m], vs, per) for m, vs in pools.items()}
        for m, vs in pools.items():
            rr = (requests_in_retention or {}).get(m, 1.0)
            decisions[m] = self.enforcer.enforce(decisions[m], vs, rr)
            for v in vs:
                v.desired = decisions[m][v.name]
            if self.actuator is not None:
                for v in vs:
                    self.actuator.scale(v, v.desired)
        self.last_decisions = decisions
        return decisions

    def fast_step(self, pools: dict[str, list[Variant]], epp_queue: dict[str, float]):
        if self.elector is not None and not self.elector.is_leader:
            return
        for m, vs in pools.items():
            d = self.sfz.check(vs, epp_queue.get(m, 0.0))
            if d is not None:
                for v in vs:
                    v.desired = d[v.name]
                    if self.actuator is not None:
                        self.actuator.scale(v, v.desired)


def _dur(s) -> float:
    s = str(s)
    mult = {"s": 1, "m": 60, "h": 3600}
    return float(s[:-1]) * mult[s[-1]] if s and s[-1] in mult else float(s)


# --------------------------------------------------------------- actuator
class ProcessActuator:
    """Single-node actuator: replicas are engine processes pinned to free GPUs."""

    def __init__(self, n_gpus: int, launch: Callable[[Variant, list[int], int], list[str]],
                 env: Optional[dict] = None):
        self.free = list(range(n_gpus))
        self.procs: dict[str, list[tuple[subprocess.Popen, list[int]]]] = {}
        self.launch = launch
        self.env = env or {}

    def scale(self, v: Variant, n: int):
        cur = self.procs.setdefault(v.name, [])
        cur[:] = [(p, g) for p, g in cur if p.poll() is None or self._release(g)]
        while len(cur) < n and len(self.free) >= v.gpus_per_replica:
            gpus = [self.free.pop(0) for _ in range(v.gpus_per_replica)]
            env = dict(os.environ, **self.env, HIP_VISIBLE_DEVICES=",".join(map(str, gpus)))
            p = subprocess.Popen(self.launch(v, gpus, len(cur)), env=env, start_new_session=True)
            cur.append((p, gpus))
        while len(cur) > n:
            p, g = cur.pop()
            self._stop(p)
            self._release(g)
        v.current = len(cur)

    def _release(self, gpus) -> bool:
        self.free.extend(gpus)
        self.free.sort()
        return False

    @staticmethod
    def _stop(p: subprocess.Popen, grace: float = 10.0):
        if p.poll() is not None:
            return
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            return
        t0 = time.time()
        while p.poll() is None and time.time() - t0 < grace:
            time.sleep(0.05)
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()

    def shutdown(self):
        for lst in self.procs.values():
            for p, g in lst:
                self._stop(p)
        self.procs.clear()


# HPA/KEDA (C32): the EPP series an external-metrics adapter maps to
# igw_queue_depth (Value target) and igw_running_requests (AverageValue target).
HPA_METRICS = {
    "igw_queue_depth": ("inference_extension_flow_control_queue_size", "Value"),
    "igw_running_requests": ("inference_objective_running_requests", "AverageValue"),
}


def hpa_desired_replicas(current: int, metric_value: float, target: float, target_type: str,
                         tolerance: float = 0.1, min_r: int = 0, max_r: int = 1 << 30) -> int:
    """Kubernetes HPA algorithm: desired = ceil(current * value / target) with a
    10% tolerance band; ``AverageValue`` divides the total by the replica count."""
    if target_type == "AverageValue":
        ratio = (metric_value / max(1, current)) / target if current else (1.0 if metric_value > 0 else 0.0)
    else:
        ratio = metric_value / target
    if current == 0:
        return max(min_r, min(max_r, 1 if metric_value > 0 else 0))
    if abs(ratio - 1.0) <= tolerance:
        return current
    return max(min_r, min(max_r, math.ceil(current * ratio)))
