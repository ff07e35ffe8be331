"""Smoke test / healthcheck for a deployed stack (reference
helpers/smoke-test/healthcheck.sh:148-421).

Checks, in order: ``/health`` (warn unless required), ``/v1/models``
(readiness, non-empty, model auto-discovery), and one inference on
``/v1/completions`` or ``/v1/chat/completions`` (``--api-mode auto`` falls
back from completions to chat) with an optional latency budget. Reports as
text or JSON (``{"endpoint", "model", "checks": {...}, "passed", "failed",
"warned", "status"}``); exit status 0 only when nothing failed.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import urllib.error
import urllib.request
from typing import Optional


def _req(url: str, payload: Optional[dict] = None, timeout: float = 30.0):
    data = json.dumps(payload).encode() if payload is not None else None
    r = urllib.request.Request(url, data=data, headers={"Content-Type": "application/json"} if data else {})
    t0 = time.monotonic()
    try:
        with urllib.request.urlopen(r, timeout=timeout) as resp:
            body = resp.read()
            return resp.status, body, (time.monotonic() - t0) * 1000
    except urllib.error.HTTPError as e:
        return e.code, e.read(), (time.monotonic() - t0) * 1000
    except (urllib.error.URLError, OSError, TimeoutError):
        return 0, b"", (time.monotonic() - t0) * 1000


def healthcheck(endpoint: str, model: Optional[str] = None, api_mode: str = "auto", prompt: str = "Hello",
                max_tokens: int = 8, max_latency_ms: int = 0, require_health: bool = False,
                timeout: float = 30.0) -> dict:
    ep = endpoint.rstrip("/")
    rep = {"endpoint": ep, "model": model, "checks": {}, "passed": 0, "failed": 0, "warned": 0}

    def mark(name, status, **kw):
        rep["checks"][name] = dict(status=status, **kw)
        rep[{"pass": "passed", "fail": "failed", "warn": "warned"}[status]] += 1

    code, _, _ = _req(ep + "/health", timeout=timeout)
    if code == 200:
        mark("health", "pass", http=code)
    else:
        mark("health", "fail" if require_health else "warn", http=code)

    code, body, _ = _req(ep + "/v1/models", timeout=timeout)
    if code != 200:
        mark("models", "fail", http=code)
    else:
        try:
            data = json.loads(body).get("data", [])
        except (json.JSONDecodeError, AttributeError):
            data = []
        if not data:
            mark("models", "fail", http=code, count=0)
        else:
            rep["model"] = model = model or data[0].get("id")
            mark("models", "pass", http=code, count=len(data))

    if not model:
        mark("inference", "fail", reason="no model id")
    else:
        paths = {"completions": ["/v1/completions"], "chat": ["/v1/chat/completions"],
                 "auto": ["/v1/completions", "/v1/chat/completions"]}[api_mode]
        for path in paths:
            if path.endswith("chat/completions"):
                payload = {"model": model, "messages": [{"role": "user", "content": prompt}],
                           "max_tokens": max_tokens, "temperature": 0}
            else:
                payload = {"model": model, "prompt": prompt, "max_tokens": max_tokens, "temperature": 0}
            code, body, lat = _req(ep + path, payload, timeout)
            if code == 200:
                break
        ok = code == 200
        try:
            out = json.loads(body)
            ok = ok and bool(out.get("choices"))
        except (json.JSONDecodeError, AttributeError):
            ok = False
        if not ok:
            mark("inference", "fail", http=code, path=path, latency_ms=round(lat))
        elif max_latency_ms and lat > max_latency_ms:
            mark("inference", "fail", http=code, path=path, latency_ms=round(lat),
                 reason=f"latency exceeds {max_latency_ms} ms")
        else:
            mark("inference", "pass", http=code, path=path, latency_ms=round(lat))
    rep["status"] = "fail" if rep["failed"] else "pass"
    return rep


def main(argv=None) -> int:
    p = argparse.ArgumentParser("llmd-healthcheck")
    p.add_argument("--endpoint", "-e", required=True)
    p.add_argument("--model", "-m")
    p.add_argument("--api-mode", choices=["auto", "completions", "chat"], default="auto")
    p.add_argument("--prompt", default="Hello")
    p.add_argument("--max-tokens", type=int, default=8)
    p.add_argument("--max-latency-ms", type=int, default=0)
    p.add_argument("--require-health", action="store_true")
    p.add_argument("--timeout", type=float, default=30.0)
    p.add_argument("--output", choices=["text", "json"], default="text")
    a = p.parse_args(argv)
    rep = healthcheck(a.endpoint, a.model, a.api_mode, a.prompt, a.max_tokens, a.max_latency_ms,
                      a.require_health, a.timeout)
    if a.output == "json":
        print(json.dumps(rep))
    else:
        for name, c in rep["checks"].items():
            print(f"[{c['status'].upper():4}] {name}: " + ", ".join(f"{k}={v}" for k, v in c.items() if k != "status"))
        print(f"{rep['passed']} passed, {rep['failed']} failed, {rep['warned']} warned -> {rep['status'].upper()}")
    return 1 if rep["failed"] else 0


if __name__ == "__main__":
    sys.exit(main())
