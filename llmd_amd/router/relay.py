"""Native router data plane: launcher for ``llmd-relay`` (csrc/relay/relay.cpp).

The reference's data plane is Envoy (C++): it holds the client and upstream
connections and relays every streamed token, while the EPP only decides
(guides/no-kubernetes-deployment/README.md:205-218; --concurrency 8 worker
threads). ``proxy --workers N`` runs that split: the EPP process serves
decisions over a Unix socket (router/workers.py EppServer) and ONE relay
process with N epoll threads (SO_REUSEPORT listeners) carries the traffic. The
Python aiohttp workers (``--data-plane python``) speak the same protocol and
remain the fallback when the executable cannot be built.
"""
from __future__ import annotations

import logging
import os
import shutil
import subprocess
from pathlib import Path
from typing import Optional

log = logging.getLogger("llmd.router.relay")


def relay_binary(build: bool = True) -> Optional[Path]:
    """Path of the built relay (building it with g++ if needed and allowed), or None.
    ``LLMD_RELAY_BIN`` overrides it (e.g. an ASan + UBSan build, tests/test_relay_sanitize.py)."""
    from llmd_amd import build as B

    if os.environ.get("LLMD_RELAY_BIN"):
        return Path(os.environ["LLMD_RELAY_BIN"])
    if B.RELAY.exists():
        try:
            return B.build_relay() if build and shutil.which("g++") else B.RELAY
        except RuntimeError:
            return B.RELAY
    if not build or shutil.which("g++") is None:
        return None
    try:
        return B.build_relay()
    except RuntimeError as e:  # noqa: PERF203 - report and fall back
        log.warning("native relay build failed: %s", e)
        return None


def spawn(uds: str, host: str, port: int, threads: int, failure_mode: str,
          binary: Optional[Path] = None) -> subprocess.Popen:
    """Start the relay process (``threads`` epoll listeners on host:port, EPP at ``uds``)."""
    b = binary or relay_binary()
    if b is None:
        raise FileNotFoundError("llmd-relay is not built (python -m llmd_amd.build relay)")
    return subprocess.Popen([str(b), "--port", str(port), "--uds", uds, "--host", host, "--threads", str(threads),
                             "--failure-mode", failure_mode])


__all__ = ["relay_binary", "spawn"]
