"""Distributed tracing (proposals/distributed-tracing.md).

Span names match the reference (``gateway.request``,
``llm_d.epp.scorer.prefix_cache``, ``llm_d.epp.pd.profile_handler.pick``,
``llm_d.pd_proxy.{request,prefill,decode}``, ``llm_request``...). W3C
``traceparent`` is parsed/propagated; sampling is parent-based with a default
ratio of 10 % (``OTEL_TRACES_SAMPLER_ARG``). If the OpenTelemetry SDK is
importable and ``OTEL_EXPORTER_OTLP_ENDPOINT`` is set, spans are exported
through it; otherwise they are kept in an in-process ring buffer
(``recent_spans()``) that tests and the debug endpoint read.
"""
from __future__ import annotations

import collections
import contextlib
import contextvars
import os
import random
import threading
import time
from dataclasses import dataclass, field
from typing import Optional

_current: contextvars.ContextVar = contextvars.ContextVar("llmd_span", default=None)
_ring: collections.deque = collections.deque(maxlen=int(os.environ.get("LLMD_TRACE_RING", "4096")))
_lock = threading.Lock()
SAMPLE_RATIO = float(os.environ.get("OTEL_TRACES_SAMPLER_ARG", "0.1"))
ENABLED = os.environ.get("LLMD_TRACING", "1") != "0"

_otel_tracer = None


def configure_otlp(endpoint: Optional[str] = None):
    """Export spans over OTLP (``--otlp-traces-endpoint`` / OTEL_EXPORTER_OTLP_ENDPOINT)
    when the OpenTelemetry SDK is importable; the in-process ring always records."""
    global _otel_tracer
    if endpoint:
        os.environ["OTEL_EXPORTER_OTLP_ENDPOINT"] = endpoint
    if not os.environ.get("OTEL_EXPORTER_OTLP_ENDPOINT"):
        return
    try:  # pragma: no cover - optional dependency
        from opentelemetry import trace as _ot

        _otel_tracer = _ot.get_tracer("llmd-amd")
    except Exception:  # noqa: BLE001
        _otel_tracer = None


configure_otlp()


@dataclass
class Span:
    name: str
    trace_id: str
    span_id: str
    parent_id: Optional[str]
    sampled: bool
    start: float = field(default_factory=time.time)
    end: Optional[float] = None
    attrs: dict = field(default_factory=dict)

    def set(self, k, v):
        self.attrs[k] = v

    @property
    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-{'01' if self.sampled else '00'}"


def parse_traceparent(tp: Optional[str]) -> Optional[tuple[str, str, bool]]:
    if not tp:
        return None
    parts = tp.strip().split("-")
    if len(parts) != 4 or len(parts[1]) != 32 or len(parts[2]) != 16:
        return None
    return parts[1], parts[2], bool(int(parts[3], 16) & 1)


def _hex(bits: int) -> str:
    """Random trace / span id (W3C ids need uniqueness, not secrecy; secrets.token_hex
    costs ~3x more on the per-request router path)."""
    return "%0*x" % (bits // 4, random.getrandbits(bits))


def current() -> Optional[Span]:
    return _current.get()


@contextlib.contextmanager
def span(name: str, attrs: Optional[dict] = None, traceparent: Optional[str] = None):
    if not ENABLED:
        yield None
        return
    parent = _current.get()
    if parent is not None:
        tid, pid, sampled = parent.trace_id, parent.span_id, parent.sampled
    else:
        ext = parse_traceparent(traceparent)
        if ext:
            tid, pid, sampled = ext
        else:
            tid, pid, sampled = _hex(128), None, random.random() < SAMPLE_RATIO
    s = Span(name, tid, _hex(64), pid, sampled, attrs=dict(attrs or {}))
    tok = _current.set(s)
    try:
        if _otel_tracer is not None and sampled:  # pragma: no cover
            with _otel_tracer.start_as_current_span(name, attributes=s.attrs):
                yield s
        else:
            yield s
    finally:
        s.end = time.time()
        _current.reset(tok)
        if sampled or os.environ.get("LLMD_TRACE_ALL") == "1":
            with _lock:
                _ring.append(s)


def recent_spans(name: Optional[str] = None) -> list[Span]:
    with _lock:
        return [s for s in _ring if name is None or s.name == name]


def inject(headers: dict):
    s = _current.get()
    if s is not None:
        headers["traceparent"] = s.traceparent
    return headers
