"""Re-export of the shared tracing helpers for router code."""
from llmd_amd.utils.tracing import current, inject, parse_traceparent, recent_spans, span  # noqa: F401
