"""Loader for the native host runtime ``llmd_amd._rt`` (builds it in-tree if missing)."""
from __future__ import annotations

_RT = None


def rt():
    global _RT
    if _RT is None:
        try:
            from llmd_amd import _rt as mod  # noqa: WPS433
        except ImportError:
            from llmd_amd.build import build_runtime

            build_runtime()
            from llmd_amd import _rt as mod  # noqa: WPS433,F811
        _RT = mod
    return _RT
