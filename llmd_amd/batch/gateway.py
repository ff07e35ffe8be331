"""Batch Gateway: OpenAI Batch API + batch processor + garbage collector
(reference docs/architecture/advanced/batch/batch-gateway.md:1-93,
guides/batch-gateway/README.md:1-180).

* API server — ``/v1/files`` (upload / list / get / content / delete) and
  ``/v1/batches`` (create / get / cancel / list); tenant isolation via a
  configurable header; input files are validated (JSONL, unique
  ``custom_id``, ``method`` POST, ``url`` == batch endpoint, ``body.model``,
  max requests per job).
* Processor — pops the earliest-deadline job from the priority queue, ingests
  the input file, builds one execution plan per model, dispatches requests to
  the router (``global`` or per-model gateway URL) under two-level concurrency
  caps (global and per-model), forwards configured pass-through headers,
  appends results / errors to output files, tracks progress, honours
  cancellation events and the completion window, then finalizes.
  On start it recovers jobs left ``in_progress`` by a crashed instance:
  partial output -> uploaded + job failed; none -> re-enqueued.
* GC — removes expired jobs and files on an interval.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import time
import uuid
from typing import Optional

from aiohttp import web
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

from .store import Store, parse_window

log = logging.getLogger("llmd.batch")

ENDPOINTS = ("/v1/chat/completions", "/v1/completions", "/v1/embeddings")
TERMINAL = ("completed", "failed", "expired", "cancelled")


class BatchMetrics:
    def __init__(self):
        r = self.registry = CollectorRegistry()
        self.requests = Counter("batch_gateway_requests_total", "Inference requests dispatched",
                                ["model", "status"], registry=r)
        self.jobs = Counter("batch_gateway_jobs_total", "Jobs by terminal status", ["status"], registry=r)
        self.job_seconds = Histogram("batch_gateway_job_processing_seconds", "Job processing time",
                                     registry=r, buckets=(1, 5, 30, 60, 300, 900, 3600, 14400, 86400))
        self.queue_wait = Histogram("batch_gateway_queue_wait_seconds", "Time from enqueue to processing",
                                    registry=r, buckets=(0.1, 1, 10, 60, 600, 3600))
        self.inflight = Gauge("batch_gateway_model_inflight_requests", "In-flight requests per model",
                              ["model"], registry=r)
        self.workers = Gauge("batch_gateway_active_jobs", "Jobs being processed", registry=r)
        self.tokens = Counter("batch_gateway_tokens_total", "Tokens in responses", ["model", "kind"], registry=r)


def _now() -> int:
    return int(time.time())


def validate_input(data: bytes, endpoint: str, max_requests: int) -> tuple[list[dict], list[dict]]:
    """Returns (requests, errors). Errors follow the OpenAI batch ``errors.data`` shape."""
    reqs, errs, seen = [], [], set()
    lines = data.decode("utf-8", errors="replace").splitlines()
    for i, line in enumerate(lines, 1):
        if not line.strip():
            continue
        try:
            r = json.loads(line)
        except json.JSONDecodeError:
            errs.append({"code": "invalid_json_line", "message": "line is not valid JSON", "line": i})
            continue
        cid = r.get("custom_id")
        if not isinstance(cid, str) or not cid:
            errs.append({"code": "missing_custom_id", "message": "custom_id is required", "line": i})
        elif cid in seen:
            errs.append({"code": "duplicate_custom_id", "message": f"duplicate custom_id {cid}", "line": i})
        if r.get("method", "POST") != "POST":
            errs.append({"code": "invalid_method", "message": "method must be POST", "line": i})
        if r.get("url") != endpoint:
            errs.append({"code": "mismatched_url", "message": f"url must be {endpoint}", "line": i})
        body = r.get("body")
        if not isinstance(body, dict) or not body.get("model"):
            errs.append({"code": "missing_model", "message": "body.model is required", "line": i})
        seen.add(cid)
        reqs.append(r)
    if not reqs and not errs:
        errs.append({"code": "empty_file", "message": "input file has no requests", "line": None})
    if len(reqs) > max_requests:
        errs.append({"code": "too_many_requests", "message": f"more than {max_requests} requests", "line": None})
    return reqs, errs


class BatchGateway:
    def __init__(self, store: Store, gateway_url: str = "http://127.0.0.1:8000",
                 model_gateways: Optional[dict] = None, tenant_header: str = "x-llm-d-tenant",
                 pass_through_headers: tuple = ("authorization",), global_concurrency: int = 256,
                 per_model_concurrency: int = 64, max_requests: int = 50000, poll_interval: float = 0.2,
                 gc_interval: float = 600.0, file_expiry_s: Optional[int] = None,
                 job_retention_s: int = 30 * 86400, request_timeout: float = 3600.0):
        self.store = store
        self.gateway_url = gateway_url.rstrip("/")
        self.model_gateways = {k: v.rstrip("/") for k, v in (model_gateways or {}).items()}
        self.tenant_header = tenant_header.lower()
        self.pass_through = tuple(h.lower() for h in pass_through_headers)
        self.global_sem_n = global_concurrency
        self.per_model_n = per_model_concurrency
        self.max_requests = max_requests
        self.poll_interval = poll_interval
        self.gc_interval = gc_interval
        self.file_expiry_s = file_expiry_s
        self.job_retention_s = job_retention_s
        self.request_timeout = request_timeout
        self.metrics = BatchMetrics()
        self._tasks: list[asyncio.Task] = []
        self._session = None
        self.active: dict[str, asyncio.Task] = {}

    # ============================================================ API server
    def _tenant(self, req: web.Request) -> str:
        return req.headers.get(self.tenant_header, "default")

    @staticmethod
    def _err(status: int, msg: str, typ: str = "invalid_request_error"):
        return web.json_response({"error": {"message": msg, "type": typ, "code": status}}, status=status)

    async def upload_file(self, req: web.Request):
        tenant = self._tenant(req)
        reader = await req.multipart()
        purpose, filename, data = None, "upload.jsonl", None
        async for part in reader:
            if part.name == "purpose":
                purpose = (await part.text()).strip()
            elif part.name == "file":
                filename = part.filename or filename
                data = await part.read(decode=False)
        if data is None:
            return self._err(400, "missing file")
        if purpose not in ("batch", "batch_output"):
            return self._err(400, "purpose must be 'batch'")
        return web.json_response(self.store.put_file(tenant, filename, purpose, bytes(data), self.file_expiry_s))

    async def list_files(self, req: web.Request):
        files = self.store.list_files(self._tenant(req), req.query.get("purpose"),
                                      int(req.query.get("limit", 10000)))
        return web.json_response({"object": "list", "data": files})

    async def get_file(self, req: web.Request):
        f = self.store.file_obj(self._tenant(req), req.match_info["id"])
        return web.json_response(f) if f else self._err(404, "file not found")

    async def file_content(self, req: web.Request):
        data = self.store.file_content(self._tenant(req), req.match_info["id"])
        if data is None:
            return self._err(404, "file not found")
        return web.Response(body=data, content_type="application/jsonl")

    async def delete_file(self, req: web.Request):
        fid = req.match_info["id"]
        ok = self.store.delete_file(self._tenant(req), fid)
        if not ok:
            return self._err(404, "file not found")
        return web.json_response({"id": fid, "object": "file", "deleted": True})

    async def create_batch(self, req: web.Request):
        tenant = self._tenant(req)
        try:
            body = await req.json()
        except json.JSONDecodeError:
            return self._err(400, "invalid JSON body")
        endpoint = body.get("endpoint")
        if endpoint not in ENDPOINTS:
            return self._err(400, f"endpoint must be one of {ENDPOINTS}")
        try:
            window = parse_window(body.get("completion_window", "24h"))
        except ValueError as e:
            return self._err(400, str(e))
        fid = body.get("input_file_id")
        if self.store.file_obj(tenant, fid) is None:
            return self._err(404, f"input file {fid} not found")
        now = _now()
        b = {"id": "batch_" + uuid.uuid4().hex, "object": "batch", "endpoint": endpoint, "errors": None,
             "input_file_id": fid, "completion_window": body.get("completion_window", "24h"),
             "status": "validating", "output_file_id": None, "error_file_id": None, "created_at": now,
             "in_progress_at": None, "expires_at": now + window, "finalizing_at": None, "completed_at": None,
             "failed_at": None, "expired_at": None, "cancelling_at": None, "cancelled_at": None,
             "request_counts": {"total": 0, "completed": 0, "failed": 0},
             "metadata": body.get("metadata"),
             "_headers": {h: req.headers[h] for h in self.pass_through if h in req.headers}}
        # synchronous validation (files are bounded by max_requests)
        reqs, errs = validate_input(self.store.file_content(tenant, fid) or b"", endpoint, self.max_requests)
        if errs:
            b.update(status="failed", failed_at=now, errors={"object": "list", "data": errs[:100]})
            self.store.put_batch(tenant, b)
            self.metrics.jobs.labels("failed").inc()
        else:
            b["request_counts"]["total"] = len(reqs)
            self.store.put_batch(tenant, b)
            self.store.enqueue(b["id"], float(b["expires_at"]))
        return web.json_response(_public(b))

    async def get_batch(self, req: web.Request):
        b = self.store.get_batch(self._tenant(req), req.match_info["id"])
        return web.json_response(_public(b)) if b else self._err(404, "batch not found")

    async def cancel_batch(self, req: web.Request):
        tenant = self._tenant(req)
        bid = req.match_info["id"]
        b = self.store.get_batch(tenant, bid)
        if b is None:
            return self._err(404, "batch not found")
        if b["status"] in TERMINAL:
            return self._err(409, f"batch is {b['status']}")
        self.store.post_event(bid, "cancel")
        b = self.store.update_batch(bid, status="cancelling", cancelling_at=_now())
        return web.json_response(_public(b))

    async def list_batches(self, req: web.Request):
        bs = self.store.list_batches(self._tenant(req), req.query.get("after"), int(req.query.get("limit", 20)))
        return web.json_response({"object": "list", "data": [_public(b) for b in bs],
                                  "first_id": bs[0]["id"] if bs else None,
                                  "last_id": bs[-1]["id"] if bs else None, "has_more": False})

    async def health(self, req):
        return web.json_response({"status": "ok", "queue": self.store.queue_len(), "active": len(self.active)})

    async def metrics_ep(self, req):
        return web.Response(body=generate_latest(self.metrics.registry), content_type="text/plain")

    def app(self) -> web.Application:
        app = web.Application(client_max_size=1 << 30)
        r = app.router
        r.add_post("/v1/files", self.upload_file)
        r.add_get("/v1/files", self.list_files)
        r.add_get("/v1/files/{id}", self.get_file)
        r.add_get("/v1/files/{id}/content", self.file_content)
        r.add_delete("/v1/files/{id}", self.delete_file)
        r.add_post("/v1/batches", self.create_batch)
        r.add_get("/v1/batches", self.list_batches)
        r.add_get("/v1/batches/{id}", self.get_batch)
        r.add_post("/v1/batches/{id}/cancel", self.cancel_batch)
        r.add_get("/health", self.health)
        r.add_get("/metrics", self.metrics_ep)
        app.on_startup.append(self._on_start)
        app.on_cleanup.append(self._on_stop)
        return app

    async def _on_start(self, app):
        self.start()

    async def _on_stop(self, app):
        await self.stop()

    # ============================================================ processor
    def start(self):
        self.recover()
        self._tasks = [asyncio.get_running_loop().create_task(self._poll_loop()),
                       asyncio.get_running_loop().create_task(self._gc_loop())]

    async def stop(self):
        for t in self._tasks + list(self.active.values()):
            t.cancel()
        for t in self._tasks + list(self.active.values()):
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        if self._session is not None:
            await self._session.close()

    def recover(self):
        """Crash recovery for jobs a previous processor left in progress."""
        for b in self.store.batches_in_status("in_progress", "finalizing", "cancelling", "validating"):
            bid, tenant = b["id"], b["_tenant"]
            if b["status"] == "validating":
                self.store.enqueue(bid, float(b["expires_at"]))
                continue
            out_path = self.store.open_output(tenant, "file-out-" + bid)
            if os.path.exists(out_path) and os.path.getsize(out_path) > 0:
                f = self.store.register_file(tenant, "file-out-" + bid, f"{bid}_output.jsonl", "batch_output",
                                             out_path)
                self.store.update_batch(bid, status="failed", failed_at=_now(), output_file_id=f["id"],
                                        errors={"object": "list", "data": [
                                            {"code": "processor_restarted",
                                             "message": "processor restarted; partial output uploaded",
                                             "line": None}]})
                self.metrics.jobs.labels("failed").inc()
            else:
                self.store.update_batch(bid, status="validating",
                                        request_counts={"completed": 0, "failed": 0})
                self.store.enqueue(bid, float(b["expires_at"]))

    async def _poll_loop(self):
        while True:
            item = self.store.dequeue()
            if item is None:
                await asyncio.sleep(self.poll_interval)
                continue
            bid, enq = item
            self.metrics.queue_wait.observe(max(0.0, time.time() - enq))
            t = asyncio.get_running_loop().create_task(self.run_job(bid))
            self.active[bid] = t
            t.add_done_callback(lambda _t, b=bid: self.active.pop(b, None))

    async def _gc_loop(self):
        while True:
            try:
                self.gc()
            except Exception:  # noqa: BLE001
                log.exception("batch gc failed")
            await asyncio.sleep(self.gc_interval)

    def gc(self, now: Optional[float] = None):
        now = now or time.time()
        for tenant, fid in self.store.expired_files(now):
            self.store.delete_file(tenant, fid)
        for b in self.store.batches_in_status(*TERMINAL):
            end = max(b.get(k) or 0 for k in ("completed_at", "failed_at", "expired_at", "cancelled_at"))
            if end and now - end > self.job_retention_s:
                self.store.delete_batch(b["id"])

    def _session_get(self):
        import aiohttp

        if self._session is None:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.request_timeout))
        return self._session

    async def run_job(self, bid: str):
        b = self.store.get_batch(None, bid)
        if b is None or b["status"] in TERMINAL:
            return
        tenant = b["_tenant"]
        if self.store.has_event(bid, "cancel"):
            self._finish(b, "cancelled", None, None)
            return
        t0 = time.time()
        self.metrics.workers.inc()
        try:
            data = self.store.file_content(tenant, b["input_file_id"]) or b""
            reqs, errs = validate_input(data, b["endpoint"], self.max_requests)
            if errs:
                self.store.update_batch(bid, status="failed", failed_at=_now(),
                                        errors={"object": "list", "data": errs[:100]})
                self.metrics.jobs.labels("failed").inc()
                return
            self.store.update_batch(bid, status="in_progress", in_progress_at=_now(),
                                    request_counts={"total": len(reqs), "completed": 0, "failed": 0})
            # per-model execution plans
            plans: dict[str, list[dict]] = {}
            for r in reqs:
                plans.setdefault(r["body"]["model"], []).append(r)
            out_fid, err_fid = "file-out-" + bid, "file-err-" + bid
            out_path = self.store.open_output(tenant, out_fid)
            err_path = self.store.open_output(tenant, err_fid)
            state = {"completed": 0, "failed": 0, "stop": None, "last_update": 0.0}
            gsem = asyncio.Semaphore(self.global_sem_n)
            with open(out_path, "w") as fo, open(err_path, "w") as fe:
                await asyncio.gather(*[self._run_plan(b, m, p, gsem, fo, fe, state) for m, p in plans.items()])
            self.store.update_batch(bid, status="finalizing", finalizing_at=_now(),
                                    request_counts={"completed": state["completed"], "failed": state["failed"]})
            out_f = self.store.register_file(tenant, out_fid, f"{bid}_output.jsonl", "batch_output", out_path) \
                if os.path.getsize(out_path) else None
            err_f = self.store.register_file(tenant, err_fid, f"{bid}_errors.jsonl", "batch_output", err_path) \
                if os.path.getsize(err_path) else None
            status = {"cancel": "cancelled", "expired": "expired"}.get(state["stop"], "completed")
            self._finish(self.store.get_batch(None, bid), status, out_f, err_f)
        finally:
            self.metrics.workers.dec()
            self.metrics.job_seconds.observe(time.time() - t0)

    def _finish(self, b, status, out_f, err_f):
        key = {"completed": "completed_at", "cancelled": "cancelled_at", "expired": "expired_at",
               "failed": "failed_at"}[status]
        self.store.update_batch(b["id"], status=status, **{key: _now()},
                                output_file_id=out_f["id"] if out_f else None,
                                error_file_id=err_f["id"] if err_f else None)
        self.metrics.jobs.labels(status).inc()

    async def _run_plan(self, b, model, plan, gsem, fo, fe, state):
        msem = asyncio.Semaphore(self.per_model_n)
        url = self.model_gateways.get(model, self.gateway_url) + b["endpoint"]
        headers = dict(b.get("_headers") or {})

        async def one(r):
            async with msem, gsem:
                if state["stop"]:
                    return
                if self.store.has_event(b["id"], "cancel"):
                    state["stop"] = "cancel"
                    return
                if time.time() > b["expires_at"]:
                    state["stop"] = "expired"
                    return
                self.metrics.inflight.labels(model).inc()
                rid = "batch_req_" + uuid.uuid4().hex
                try:
                    body = dict(r["body"], stream=False)
                    async with self._session_get().post(url, json=body,
                                                        headers=dict(headers, **{"x-request-id": rid})) as resp:
                        try:
                            rb = await resp.json(content_type=None)
                        except (json.JSONDecodeError, ValueError):
                            rb = {"error": {"message": (await resp.text())[:500]}}
                        status = resp.status
                except Exception as e:  # noqa: BLE001
                    status, rb = 0, {"error": {"message": str(e)}}
                finally:
                    self.metrics.inflight.labels(model).dec()
                if status == 200:
                    fo.write(json.dumps({"id": rid, "custom_id": r["custom_id"],
                                         "response": {"status_code": 200, "request_id": rid, "body": rb},
                                         "error": None}) + "\n")
                    state["completed"] += 1
                    u = rb.get("usage") or {}
                    self.metrics.tokens.labels(model, "prompt").inc(u.get("prompt_tokens", 0))
                    self.metrics.tokens.labels(model, "completion").inc(u.get("completion_tokens", 0))
                    self.metrics.requests.labels(model, "success").inc()
                else:
                    err = (rb or {}).get("error") or {}
                    fe.write(json.dumps({"id": rid, "custom_id": r["custom_id"],
                                         "response": {"status_code": status, "request_id": rid, "body": rb}
                                         if status else None,
                                         "error": {"code": str(err.get("code", status or "connection_error")),
                                                   "message": err.get("message", "")}}) + "\n")
                    state["failed"] += 1
                    self.metrics.requests.labels(model, "failure").inc()
                now = time.time()
                if now - state["last_update"] > 0.5:
                    state["last_update"] = now
                    self.store.update_batch(b["id"], request_counts={"completed": state["completed"],
                                                                     "failed": state["failed"]})

        await asyncio.gather(*[one(r) for r in plan])


def _public(b: dict) -> dict:
    return {k: v for k, v in b.items() if not k.startswith("_")}


def main(argv=None):
    p = argparse.ArgumentParser("llmd-batch-gateway")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8081)
    p.add_argument("--root", default="/var/lib/llmd-batch")
    p.add_argument("--gateway-url", default="http://127.0.0.1:8000")
    p.add_argument("--model-gateways", default="{}", help="JSON {model: url}")
    p.add_argument("--tenant-header", default="x-llm-d-tenant")
    p.add_argument("--pass-through-headers", default="authorization")
    p.add_argument("--global-concurrency", type=int, default=256)
    p.add_argument("--per-model-concurrency", type=int, default=64)
    p.add_argument("--max-requests", type=int, default=50000)
    a = p.parse_args(argv)
    gw = BatchGateway(Store(a.root), a.gateway_url, json.loads(a.model_gateways), a.tenant_header,
                      tuple(h for h in a.pass_through_headers.split(",") if h), a.global_concurrency,
                      a.per_model_concurrency, a.max_requests)
    web.run_app(gw.app(), host=a.host, port=a.port, access_log=None)


if __name__ == "__main__":
    main()
