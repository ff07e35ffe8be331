"""EPP HTTP header contract (docs/api-reference/epp-http-headers.md:9-66).

Canonical ``x-llm-d-*`` names win over deprecated aliases; all lookups are
case-insensitive.
"""
from __future__ import annotations

from typing import Optional

OBJECTIVE = "x-llm-d-inference-objective"
FAIRNESS_ID = "x-llm-d-inference-fairness-id"
MODEL_REWRITE = "x-llm-d-model-name-rewrite"
SLO_TTFT = "x-llm-d-slo-ttft-ms"
SLO_TPOT = "x-llm-d-slo-tpot-ms"
DROPPED_REASON = "x-llm-d-request-dropped-reason"
# internal / GAIE protocol headers
DESTINATION = "x-gateway-destination-endpoint"
PREFILLER = "x-prefiller-host-port"
ENCODER = "x-encoder-hosts-ports"
REQUEST_ID = "x-request-id"
TRACEPARENT = "traceparent"

ALIASES = {
    FAIRNESS_ID: "x-gateway-inference-fairness-id",
    OBJECTIVE: "x-gateway-inference-objective",
    MODEL_REWRITE: "x-gateway-model-name-rewrite",
    SLO_TTFT: "x-slo-ttft-ms",
    SLO_TPOT: "x-slo-tpot-ms",
}

DEFAULT_FAIRNESS_ID = "default-flow"

# dropped-reason values
REJECTED_SATURATED = "rejected-saturated"
REJECTED_TTL = "rejected-ttl-expired"
REJECTED_CANCELLED = "rejected-context-cancelled"
EVICTED = "evicted"


def lookup(headers, canonical: str) -> Optional[str]:
    """Canonical header first, then its deprecated alias (case-insensitive)."""
    v = _get(headers, canonical)
    if v is not None and v != "":
        return v
    alias = ALIASES.get(canonical)
    if alias:
        v = _get(headers, alias)
        if v is not None and v != "":
            return v
    return None


def _get(headers, k):
    if headers is None:
        return None
    try:
        v = headers.get(k)
        if v is None and not getattr(headers, "case_insensitive", False):
            low = k.lower()
            for hk, hv in headers.items():
                if hk.lower() == low:
                    return hv
        return v
    except AttributeError:
        return None


def float_header(headers, canonical: str) -> Optional[float]:
    v = lookup(headers, canonical)
    if v is None:
        return None
    try:
        return float(v)
    except ValueError:
        return None
