"""Plugin framework: roles, registry and auto-wiring by implemented interface
(docs/architecture/core/router/epp/configuration.md:38-56, 189-216).

A plugin class declares the roles it implements by subclassing the role base
classes below; the config loader binds Admitters, DataProducers, PreRequest
and Response processors automatically, and validates that profile references
resolve to Filters / Scorers / Pickers.
"""
from __future__ import annotations

from typing import Any, Callable, Optional

from ..types import Endpoint, InferenceRequest, ProfileRunResult, SchedulingResult

REGISTRY: dict[str, type] = {}
DEPRECATED_ALIASES: dict[str, str] = {}


def register(type_name: str, *aliases: str):
    def deco(cls):
        REGISTRY[type_name] = cls
        cls.plugin_type = type_name
        for a in aliases:
            REGISTRY[a] = cls
            DEPRECATED_ALIASES[a] = type_name
        return cls

    return deco


class Plugin:
    plugin_type = "plugin"

    def __init__(self, name: str, params: Optional[dict] = None, ctx: Any = None):
        self.name = name
        self.params = dict(params or {})
        self.ctx = ctx  # the EPP runtime (datastore, metrics, other plugins)

    def p(self, key: str, default=None):
        return self.params.get(key, default)

    async def start(self):
        """Optional async startup (subscribers, pollers)."""

    async def stop(self):
        pass

    def __repr__(self):
        return f"<{self.plugin_type} {self.name}>"


# ---------------------------------------------------------------- scheduling roles
class Filter(Plugin):
    def filter(self, req: InferenceRequest, eps: list[Endpoint]) -> list[Endpoint]:
        raise NotImplementedError


class Scorer(Plugin):
    def score(self, req: InferenceRequest, eps: list[Endpoint]) -> dict[str, float]:
        """endpoint key -> score in [0, 1]"""
        raise NotImplementedError


class Picker(Plugin):
    def pick(self, req: InferenceRequest, scored: list[tuple[Endpoint, float]]) -> list[Endpoint]:
        raise NotImplementedError


class ProfileHandler(Plugin):
    def pick_profiles(self, req: InferenceRequest, profiles: dict, results: dict) -> list[str]:
        raise NotImplementedError

    def process_results(self, req: InferenceRequest, results: dict[str, ProfileRunResult]) -> SchedulingResult:
        raise NotImplementedError


# ---------------------------------------------------------------- request control roles
class Parser(Plugin):
    def parse(self, path: str, body: bytes, headers) -> InferenceRequest:
        raise NotImplementedError

    def parse_usage(self, chunk: dict) -> Optional[dict]:
        return chunk.get("usage") if isinstance(chunk, dict) else None


class DataProducer(Plugin):
    async def produce(self, req: InferenceRequest, eps: list[Endpoint]) -> None:
        raise NotImplementedError


class Admitter(Plugin):
    def admit(self, req: InferenceRequest, eps: list[Endpoint]) -> Optional[tuple[int, str]]:
        """None to admit, or (http_status, reason) to reject."""
        raise NotImplementedError


class PreRequest(Plugin):
    def pre_request(self, req: InferenceRequest, result: SchedulingResult) -> None:
        raise NotImplementedError


class ResponseProcessor(Plugin):
    def on_response_headers(self, req: InferenceRequest, ep: Endpoint, status: int, headers) -> None:
        pass

    def on_response_chunk(self, req: InferenceRequest, ep: Endpoint, chunk: bytes, t: float) -> None:
        pass

    def on_response_complete(self, req: InferenceRequest, ep: Endpoint, info: dict) -> None:
        pass


# ---------------------------------------------------------------- flow control roles
class FairnessPolicy(Plugin):
    def pick_flow(self, band) -> Optional[Any]:
        raise NotImplementedError


class OrderingPolicy(Plugin):
    def key(self, item) -> Any:
        raise NotImplementedError


class SaturationDetector(Plugin):
    def saturation(self, eps: list[Endpoint]) -> float:
        """>= 1.0 means saturated."""
        raise NotImplementedError


# ---------------------------------------------------------------- data layer roles
class DataSource(Plugin):
    pass


class Extractor(Plugin):
    def extract(self, ep: Endpoint, data: Any) -> None:
        raise NotImplementedError


class Decider(Plugin):
    def should_disaggregate(self, req: InferenceRequest, decode_ep: Endpoint) -> bool:
        raise NotImplementedError


def create(type_name: str, name: Optional[str], params: Optional[dict], ctx) -> Plugin:
    if type_name not in REGISTRY:
        raise ValueError(f"unknown plugin type {type_name!r}")
    return REGISTRY[type_name](name or type_name, params, ctx)


def roles(p: Plugin) -> set[str]:
    out = set()
    for cls, r in ((Filter, "filter"), (Scorer, "scorer"), (Picker, "picker"),
                   (ProfileHandler, "profile-handler"), (Parser, "parser"), (DataProducer, "data-producer"),
                   (Admitter, "admitter"), (PreRequest, "pre-request"), (ResponseProcessor, "response-processor"),
                   (FairnessPolicy, "fairness"), (OrderingPolicy, "ordering"),
                   (SaturationDetector, "saturation-detector"), (DataSource, "data-source"),
                   (Extractor, "extractor"), (Decider, "decider")):
        if isinstance(p, cls):
            out.add(r)
    return out
