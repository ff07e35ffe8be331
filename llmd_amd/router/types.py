"""Core router data types: endpoints, requests, scheduling results.

Mirrors the EPP framework concepts (docs/architecture/core/router/epp/
scheduling.md:46-60, datalayer.md:40-48): an Endpoint is one (pod, port)
model-server engine with a thread-safe attribute map filled by the data
layer; an InferenceRequest is the parsed, enriched request the plugins see.
"""
from __future__ import annotations

import itertools
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Optional

_req_ids = itertools.count(1)


class Attributes:
    """Thread-safe typed attribute map stored on each endpoint."""

    def __init__(self):
        self._d: dict[str, Any] = {}
        self._lock = threading.Lock()

    def get(self, k: str, default=None):
        # a single dict read is atomic under the GIL; writers still lock
        return self._d.get(k, default)

    def put(self, k: str, v: Any):
        with self._lock:
            self._d[k] = v
            ATTR_VERSION[0] += 1

    def update(self, d: dict):
        with self._lock:
            self._d.update(d)
            ATTR_VERSION[0] += 1

    def snapshot(self) -> dict:
        with self._lock:
            return dict(self._d)


# bumped by every Attributes write: per-request consumers of slowly changing endpoint attributes
# (the prefix producer's LRU auto-tune) skip their scan while nothing changed
ATTR_VERSION = [0]

# standard metric attribute keys (core-metrics-extractor output)
WAITING = "WaitingQueueSize"
RUNNING = "RunningRequestsSize"
KV_USAGE = "KVCacheUsagePercent"
BLOCK_SIZE = "BlockSize"
NUM_GPU_BLOCKS = "NumGPUBlocks"
MAX_LORA = "MaxActiveModels"
ACTIVE_LORAS = "ActiveModels"
WAITING_LORAS = "WaitingModels"
METRICS_TS = "MetricsUpdateTime"


@dataclass(eq=False)
class Endpoint:
    name: str                       # pod name (or synthetic)
    address: str                    # ip
    port: int
    namespace: str = "default"
    labels: dict = field(default_factory=dict)
    metrics_port: Optional[int] = None
    attrs: Attributes = field(default_factory=Attributes)
    healthy: bool = True

    key: str = field(init=False, repr=False)  # "ip:port", read per scorer per endpoint: a plain attribute

    def __post_init__(self):
        self.key = f"{self.address}:{self.port}"

    @property
    def role(self) -> str:
        return self.labels.get("llm-d.ai/role", "prefill-decode")

    def metric(self, k: str, default=0.0):
        return self.attrs._d.get(k, default)  # scorers call this per endpoint: skip one frame

    def __repr__(self):
        return f"Endpoint({self.name}@{self.key})"

    def __hash__(self):
        return hash(self.key)


class CIHeaders(dict):
    """Case-insensitive header mapping (keys stored lower-case)."""

    case_insensitive = True  # headers._get: a miss is final, no scan

    def __init__(self, d=None):
        super().__init__()
        for k, v in (d or {}).items():
            self[k] = v

    def __setitem__(self, k, v):
        super().__setitem__(k.lower(), v)

    def __getitem__(self, k):
        return super().__getitem__(k.lower())

    def get(self, k, default=None):
        return super().get(k.lower(), default)

    def __contains__(self, k):
        return super().__contains__(k.lower())

    def pop(self, k, *a):
        return super().pop(k.lower(), *a)


@dataclass
class InferenceRequest:
    path: str
    body: dict
    headers: CIHeaders
    raw_size: int = 0
    request_id: str = field(default_factory=lambda: f"epp-{next(_req_ids)}")
    model: str = ""
    target_model: str = ""
    objective: Optional[str] = None
    priority: int = 0
    fairness_id: str = "default-flow"
    slo_ttft_ms: Optional[float] = None
    slo_tpot_ms: Optional[float] = None
    prompt: str = ""                      # flattened text used for approximate hashing
    token_ids: Optional[list[int]] = None  # exact tokens (token-producer)
    mm_assets: list = field(default_factory=list)  # (asset hash, estimated tokens) per image
    stream: bool = False
    data: dict = field(default_factory=dict)  # producer outputs
    arrival: float = field(default_factory=time.monotonic)
    deadline: Optional[float] = None

    @property
    def sheddable(self) -> bool:
        return self.priority < 0


@dataclass
class ProfileRunResult:
    targets: list[Endpoint]
    scores: dict = field(default_factory=dict)  # endpoint key -> aggregate score


@dataclass
class SchedulingResult:
    primary_profile: str
    profile_results: dict[str, ProfileRunResult]
    headers: dict = field(default_factory=dict)  # headers to add to the upstream request

    @property
    def target(self) -> Optional[Endpoint]:
        r = self.profile_results.get(self.primary_profile)
        return r.targets[0] if r and r.targets else None


class SchedulingError(Exception):
    def __init__(self, status: int, msg: str, reason: str = ""):
        super().__init__(msg)
        self.status = status
        self.reason = reason
