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


class Span:
    """One span. ``span_id`` is drawn lazily (the first time it is read: a child span,
    ``traceparent`` injection, an exporter), so the unsampled majority of spans on the
    router's per-request path cost no id generation."""

    __slots__ = ("name", "trace_id", "_span_id", "parent_id", "sampled", "start", "end", "attrs")

    def __init__(self, name: str, trace_id: str, span_id: Optional[str], parent_id: Optional[str], sampled: bool,
                 start: Optional[float] = None, end: Optional[float] = None, attrs: Optional[dict] = None):
        self.name = name
        self.trace_id = trace_id
        self._span_id = span_id
        self.parent_id = parent_id
        self.sampled = sampled
        self.start = time.time() if start is None else start
        self.end = end
        self.attrs = {} if attrs is None else attrs

    @property
    def span_id(self) -> str:
        if self._span_id is None:
            self._span_id = _hex(64)
        return self._span_id

    def set(self, k, v):
        self.attrs[k] = v

    @property
    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-{'01' if self.sampled else '00'}"

    def __repr__(self):
        return f"Span({self.name!r}, trace={self.trace_id}, span={self.span_id}, parent={self.parent_id})"


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


_TRACE_ALL = os.environ.get("LLMD_TRACE_ALL") == "1"


class _SpanCtx:
    """``with span(...) as s``: a plain context-manager object (a generator-based
    contextmanager costs several microseconds per use; the EPP opens ~6 spans per request)."""

    __slots__ = ("name", "attrs", "tp", "s", "tok", "ot")

    def __init__(self, name, attrs, tp):
        self.name, self.attrs, self.tp = name, attrs, tp
        self.s = self.tok = self.ot = None

    def __enter__(self):
        if not ENABLED:
            return None
        parent = _current.get()
        if parent is not None:
            if not parent.sampled and not _TRACE_ALL and _otel_tracer is None:
                # a child of an unsampled trace is never recorded or exported: skip the Span (ids,
                # attrs, context var) - the EPP opens several per decision (~1 us each)
                return None
            tid, pid, sampled = parent.trace_id, parent.span_id, parent.sampled
        else:
            ext = parse_traceparent(self.tp)
            if ext:
                tid, pid, sampled = ext
            else:
                tid, pid, sampled = _hex(128), None, random.random() < SAMPLE_RATIO
        s = self.s = Span(self.name, tid, None, pid, sampled, attrs=dict(self.attrs) if self.attrs else None)
        self.tok = _current.set(s)
        if _otel_tracer is not None and sampled:  # pragma: no cover
            self.ot = _otel_tracer.start_as_current_span(self.name, attributes=s.attrs)
            self.ot.__enter__()
        return s

    def __exit__(self, et, ev, tb):
        s = self.s
        if s is None:
            return False
        if self.ot is not None:  # pragma: no cover
            self.ot.__exit__(et, ev, tb)
        s.end = time.time()
        _current.reset(self.tok)
        if s.sampled or _TRACE_ALL:
            with _lock:
                _ring.append(s)
        return False


def span(name: str, attrs: Optional[dict] = None, traceparent: Optional[str] = None) -> _SpanCtx:
    return _SpanCtx(name, attrs, traceparent)


def recent_spans(name: Optional[str] = None) -> list[Span]:
    with _lock:
        return [s for s in _ring if name is None or s.name == name]


def inject(headers: dict):
    s = _current.get()
    if s is not None:
        headers["traceparent"] = s.traceparent
    return headers
