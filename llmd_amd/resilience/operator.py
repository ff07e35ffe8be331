"""Inference Resilience Operator (IRO) for one node (the design of
proposals/inference-resilience-operator.md:66-256).

IRO sits between the infrastructure layer (whatever detects hardware faults)
and the engines. It has two input channels with separate duties:

* ``RecoveryRequest`` objects (infrastructure initiated). The infrastructure
  recovery controller creates one per hardware fault, with the resolved
  ``requestedAction``; IRO coordinates the engine side and restores capacity
  when ``status.phase`` reaches ``Completed``:

  ====================  =====  ===========================================
  requestedAction       track  engine side
  ====================  =====  ===========================================
  RESET_DEVICE          A      pause -> (device reset) -> resume
  REBOOT_NODE           B      pause -> (node reboot) -> resume
  REPLACE_NODE          C      scale down -> (replacement) -> scale up
  ====================  =====  ===========================================

  ``status.conditions[EngineReadyForRecovery]`` is set once the engine is
  paused / scaled down, so a controller that gates on it can wait (the
  proposal's open question: both gated and un-gated controllers work). A
  ``Failed`` phase degrades the engines: they stay out of routing.
* ``vllm_fault`` events (engine initiated, ``fault@<model>`` topic on the KV
  event channel, see ``serving/api_server.py``). A fault with no
  ``RecoveryRequest`` covering the engine is transient: IRO tells the engine
  to ``retry``; after ``maxRetries`` within ``retryWindow`` it gives up and
  takes the engine out of routing.

On one node the CRD store is a directory of YAML objects (``kind:
RecoveryRequest``; an infrastructure controller writes them, or POSTs to
``/apis/recoveryrequests`` here), "scale down" removes the engine's endpoints
from the router's file-discovery ``endpoints.yaml`` (atomic rename; the removed
entries are kept in the request's status so a restarted operator can put them
back), and the rank topology map (``nodeName`` + ``deviceID`` -> engines) comes
from the config. Engines in one ``group`` (the DP ranks of a wide-EP
deployment, which step in lockstep and share the EP all-to-all) are affected
together: a fault on any device of the group pauses all of its ranks, since the
EP world cannot shrink in place (the elastic-EP RFCs the proposal cites are not
merged upstream either).

The ``EngineAdapter`` interface is the proposal's (FaultEvents, EngineStatus,
PauseEngine, ResumeEngine, ScaleDown, ScaleUp); ``LLMDEngineAdapter`` drives
this repo's API server (``/fault_tolerance/status``, ``/fault_tolerance/apply``).

  python -m llmd_amd.resilience.operator --config iro.yaml
  python -m llmd_amd.resilience.operator request --store DIR --node node-0 --device 3 --action RESET_DEVICE
  python -m llmd_amd.resilience.operator complete --store DIR NAME [--failed]
"""
from __future__ import annotations

import argparse
import asyncio
import fcntl
import logging
import os
import time
import uuid
from collections import defaultdict, deque
from dataclasses import dataclass, field
from typing import Callable, Optional

import aiohttp
import yaml
from aiohttp import web

log = logging.getLogger("llmd.iro")

TRACKS = {"RESET_DEVICE": "A", "REBOOT_NODE": "B", "REPLACE_NODE": "C"}
PHASES = ("Pending", "InProgress", "Completed", "Failed")
# IRO's own progress on a request (status.iroState)
S_NEW, S_PAUSED, S_SCALED_DOWN, S_RECOVERED, S_DEGRADED = "", "EnginePaused", "EngineScaledDown", "Recovered", "Degraded"
TERMINAL = (S_RECOVERED, S_DEGRADED)
API_VERSION = "llm-d.ai/v1alpha1"


# ------------------------------------------------------------------ CRD store
@dataclass
class RecoveryRequest:
    name: str
    node_name: str
    requested_action: str
    device_id: Optional[int] = None
    error_code: Optional[str] = None
    phase: str = "Pending"
    conditions: dict = field(default_factory=dict)   # type -> "True"/"False"
    iro_state: str = S_NEW
    engines: list = field(default_factory=list)      # engines IRO acted on
    removed_endpoints: list = field(default_factory=list)
    message: str = ""

    @classmethod
    def from_obj(cls, d: dict) -> "RecoveryRequest":
        if d.get("kind") != "RecoveryRequest":
            raise ValueError(f"not a RecoveryRequest: kind={d.get('kind')!r}")
        spec, st = d.get("spec") or {}, d.get("status") or {}
        act = spec.get("requestedAction")
        if act not in TRACKS:
            raise ValueError(f"requestedAction must be one of {sorted(TRACKS)}, got {act!r}")
        if not spec.get("nodeName"):
            raise ValueError("spec.nodeName is required")
        phase = st.get("phase", "Pending")
        if phase not in PHASES:
            raise ValueError(f"status.phase must be one of {PHASES}, got {phase!r}")
        dev = spec.get("deviceID")
        return cls(name=d["metadata"]["name"], node_name=str(spec["nodeName"]), requested_action=act,
                   device_id=None if dev is None else int(dev), error_code=spec.get("errorCode"),
                   phase=phase, conditions={c["type"]: c["status"] for c in st.get("conditions", [])},
                   iro_state=st.get("iroState", S_NEW), engines=list(st.get("engines", [])),
                   removed_endpoints=list(st.get("removedEndpoints", [])), message=st.get("message", ""))

    def to_obj(self) -> dict:
        spec = {"nodeName": self.node_name, "requestedAction": self.requested_action}
        if self.device_id is not None:
            spec["deviceID"] = self.device_id
        if self.error_code is not None:
            spec["errorCode"] = self.error_code
        st = {"phase": self.phase, "iroState": self.iro_state,
              "conditions": [{"type": k, "status": v} for k, v in sorted(self.conditions.items())]}
        if self.engines:
            st["engines"] = self.engines
        if self.removed_endpoints:
            st["removedEndpoints"] = self.removed_endpoints
        if self.message:
            st["message"] = self.message
        return {"apiVersion": API_VERSION, "kind": "RecoveryRequest", "metadata": {"name": self.name},
                "spec": spec, "status": st}

    @property
    def track(self) -> str:
        return TRACKS[self.requested_action]

    @property
    def active(self) -> bool:
        return self.iro_state not in TERMINAL


class RecoveryStore:
    """RecoveryRequest objects as ``<name>.yaml`` in one directory. Writers
    (the infrastructure controller owns ``spec`` and ``status.phase``, IRO the
    rest of ``status``) update under an flock with an atomic rename, so a
    reader never sees a torn object and neither side loses the other's field."""

    def __init__(self, root: str):
        self.root = root
        os.makedirs(root, exist_ok=True)
        self._lock_path = os.path.join(root, ".lock")

    def _path(self, name: str) -> str:
        if not name or "/" in name or name.startswith("."):
            raise ValueError(f"bad object name {name!r}")
        return os.path.join(self.root, f"{name}.yaml")

    def _locked(self):
        f = open(self._lock_path, "a")
        fcntl.flock(f, fcntl.LOCK_EX)
        return f

    def _write(self, rr: RecoveryRequest):
        p = self._path(rr.name)
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            yaml.safe_dump(rr.to_obj(), f, sort_keys=False)
        os.replace(tmp, p)

    def list(self) -> list[RecoveryRequest]:
        out = []
        for fn in sorted(os.listdir(self.root)):
            if not fn.endswith(".yaml"):
                continue
            try:
                with open(os.path.join(self.root, fn)) as f:
                    out.append(RecoveryRequest.from_obj(yaml.safe_load(f) or {}))
            except (OSError, ValueError, KeyError, TypeError, yaml.YAMLError) as e:
                log.warning("skipping %s: %s", fn, e)
        return out

    def get(self, name: str) -> Optional[RecoveryRequest]:
        try:
            with open(self._path(name)) as f:
                return RecoveryRequest.from_obj(yaml.safe_load(f) or {})
        except FileNotFoundError:
            return None

    def create(self, obj: dict) -> RecoveryRequest:
        obj = dict(obj)
        obj.setdefault("apiVersion", API_VERSION)
        obj.setdefault("kind", "RecoveryRequest")
        md = dict(obj.get("metadata") or {})
        md.setdefault("name", f"rr-{uuid.uuid4().hex[:8]}")
        obj["metadata"] = md
        rr = RecoveryRequest.from_obj(obj)
        with self._locked():
            if os.path.exists(self._path(rr.name)):
                raise FileExistsError(rr.name)
            self._write(rr)
        return rr

    def update(self, name: str, fn: Callable[[RecoveryRequest], None]) -> Optional[RecoveryRequest]:
        """Read-modify-write of one object under the store lock."""
        with self._locked():
            rr = self.get(name)
            if rr is None:
                return None
            fn(rr)
            self._write(rr)
            return rr

    def set_phase(self, name: str, phase: str) -> Optional[RecoveryRequest]:
        if phase not in PHASES:
            raise ValueError(f"phase must be one of {PHASES}")
        return self.update(name, lambda rr: setattr(rr, "phase", phase))


# ------------------------------------------------------------------ engines
class EngineAdapter:
    """The proposal's EngineAdapter operations (inference-resilience-operator.md:170-186)."""

    def __init__(self, name: str, node_name: str, devices: list[int], endpoints: list[dict], group: str = ""):
        self.name, self.node_name, self.devices = name, node_name, list(devices)
        self.endpoints = endpoints  # router endpoints this engine serves (address, port)
        self.group = group or name

    async def status(self) -> dict:
        raise NotImplementedError

    async def pause(self):
        raise NotImplementedError

    async def resume(self):
        raise NotImplementedError

    async def retry(self):
        raise NotImplementedError

    async def scale_down(self):
        """Stop serving: the operator has already taken the engine out of routing."""
        await self.pause()

    async def scale_up(self):
        await self.resume()

    def fault_events(self, on_fault: Callable[["EngineAdapter", dict], None]):
        """Start delivering engine-initiated fault events; returns a stopper or None."""
        return None


class LLMDEngineAdapter(EngineAdapter):
    """This repo's API server: ``/fault_tolerance/{status,apply}`` over HTTP and
    ``vllm_fault`` events on the engine's KV-event publisher."""

    def __init__(self, name, node_name, devices, endpoints, url: str, fault_endpoint: Optional[str] = None,
                 group: str = "", timeout: float = 10.0):
        super().__init__(name, node_name, devices, endpoints, group)
        self.url = url.rstrip("/")
        self.fault_endpoint = fault_endpoint
        self.timeout = aiohttp.ClientTimeout(total=timeout)
        self._sub = None

    async def status(self) -> dict:
        try:
            async with aiohttp.ClientSession(timeout=self.timeout) as s:
                async with s.get(self.url + "/fault_tolerance/status") as r:
                    return await r.json()
        except (aiohttp.ClientError, asyncio.TimeoutError, OSError) as e:
            return {"status": "unreachable", "faults": [{"kind": "unreachable", "detail": repr(e)}]}

    async def _apply(self, action: str, **kw):
        async with aiohttp.ClientSession(timeout=self.timeout) as s:
            async with s.post(self.url + "/fault_tolerance/apply", json={"action": action, **kw}) as r:
                if r.status != 200:
                    raise RuntimeError(f"{self.name}: {action} -> HTTP {r.status}: {await r.text()}")

    async def pause(self):
        await self._apply("pause")

    async def resume(self):
        await self._apply("resume")

    async def retry(self):
        await self._apply("retry")

    def fault_events(self, on_fault):
        if not self.fault_endpoint:
            return None
        from llmd_amd.serving.kv_events import KVEventSubscriber

        def on_batch(topic, batch):
            for ev in batch.get("events", []):
                if isinstance(ev, dict) and ev.get("type") == "vllm_fault":
                    on_fault(self, ev)

        self._sub = KVEventSubscriber(self.fault_endpoint, on_batch, topic_filter="fault@").start()
        return self._sub


# ------------------------------------------------------------------ reconciler
def _ep_key(e: dict) -> tuple:
    return (str(e.get("address", "127.0.0.1")), int(e["port"]))


class ResilienceOperator:
    def __init__(self, cfg: dict, adapters: Optional[list[EngineAdapter]] = None):
        self.cfg = cfg
        self.store = RecoveryStore(cfg["recoveryRequestsDir"])
        self.endpoints_file = cfg.get("endpointsFile")
        self.interval = float(cfg.get("interval", 1.0))
        self.recover_timeout = float(cfg.get("recoverTimeout", 120.0))
        self.max_retries = int(cfg.get("maxRetries", 3))
        self.retry_window = float(cfg.get("retryWindow", 300.0))
        self.poll_status = bool(cfg.get("pollEngineStatus", True))
        self.adapters: list[EngineAdapter] = adapters if adapters is not None else \
            [self._adapter(e) for e in cfg.get("engines", [])]
        self.by_name = {a.name: a for a in self.adapters}
        self.actions: dict[tuple, int] = defaultdict(int)        # (engine, action) -> count
        self.transient: dict[str, deque] = defaultdict(deque)    # engine -> fault timestamps
        self.degraded: set[str] = set()                          # engines IRO gave up on (no request)
        self.degraded_eps: dict[str, list] = {}
        self._faulted: set[str] = set()
        self._lock = asyncio.Lock()
        self._subs = []
        self._task: Optional[asyncio.Task] = None

    @staticmethod
    def _adapter(e: dict) -> EngineAdapter:
        url = e["url"]
        host_port = url.split("://", 1)[-1].rstrip("/")
        host, _, port = host_port.rpartition(":")
        eps = e.get("endpoints") or [{"address": host, "port": int(port)}]
        return LLMDEngineAdapter(e["name"], str(e.get("nodeName", "localhost")), e.get("devices", []), eps,
                                 url=url, fault_endpoint=e.get("faultEvents"), group=e.get("group", ""))

    # ---------------------------------------------------------- topology
    def affected(self, rr: RecoveryRequest) -> list[EngineAdapter]:
        """Rank topology map: engines on ``nodeName`` using ``deviceID`` (all of
        the node's engines if no device), widened to their whole groups."""
        hit = [a for a in self.adapters if a.node_name == rr.node_name
               and (rr.device_id is None or rr.device_id in a.devices)]
        groups = {a.group for a in hit}
        return [a for a in self.adapters if a.group in groups]

    # ---------------------------------------------------------- routing
    def _read_endpoints(self) -> list[dict]:
        try:
            with open(self.endpoints_file) as f:
                return list((yaml.safe_load(f) or {}).get("endpoints") or [])
        except FileNotFoundError:
            return []

    def _write_endpoints_file(self, eps: list[dict]):
        tmp = self.endpoints_file + ".iro.tmp"
        with open(tmp, "w") as f:
            yaml.safe_dump({"endpoints": eps}, f, sort_keys=False)
        os.replace(tmp, self.endpoints_file)

    def remove_from_routing(self, engines: list[EngineAdapter]) -> list[dict]:
        if not self.endpoints_file:
            return []
        keys = {_ep_key(e) for a in engines for e in a.endpoints}
        eps = self._read_endpoints()
        removed = [e for e in eps if _ep_key(e) in keys]
        if removed:
            self._write_endpoints_file([e for e in eps if _ep_key(e) not in keys])
        return removed

    def restore_routing(self, removed: list[dict]):
        if not self.endpoints_file or not removed:
            return
        eps = self._read_endpoints()
        have = {_ep_key(e) for e in eps}
        eps += [e for e in removed if _ep_key(e) not in have]
        self._write_endpoints_file(eps)

    # ---------------------------------------------------------- actions
    async def _do(self, a: EngineAdapter, action: str):
        self.actions[(a.name, action)] += 1
        log.info("engine %s: %s", a.name, action)
        await getattr(a, action)()

    async def _each(self, engines, action) -> list[str]:
        errs = []
        res = await asyncio.gather(*(self._do(a, action) for a in engines), return_exceptions=True)
        for a, r in zip(engines, res):
            if isinstance(r, BaseException):
                errs.append(f"{a.name}: {action} failed: {r}")
        return errs

    async def _wait_healthy(self, engines) -> bool:
        deadline = time.monotonic() + self.recover_timeout
        while time.monotonic() < deadline:
            sts = await asyncio.gather(*(a.status() for a in engines))
            if all(s.get("status") == "healthy" for s in sts):
                return True
            await asyncio.sleep(min(0.5, self.interval))
        return False

    async def reconcile_one(self, rr: RecoveryRequest):
        if not rr.active:
            return
        engines = [self.by_name[n] for n in rr.engines if n in self.by_name] if rr.engines else self.affected(rr)
        names = [a.name for a in engines]
        if rr.iro_state == S_NEW and rr.phase in ("Pending", "InProgress"):
            if not engines:
                self.store.update(rr.name, lambda r: (setattr(r, "iro_state", S_DEGRADED),
                                                      setattr(r, "message", "no engine on that node/device")))
                return
            grouped = any(sum(b.group == a.group for b in self.adapters) > 1 for a in engines)
            if rr.track == "C" and not grouped:
                removed = self.remove_from_routing(engines)
                errs = await self._each(engines, "scale_down")
                state = S_SCALED_DOWN
            else:  # A / B, or C on a lockstep group (cannot shrink in place): pause every rank
                removed = []
                errs = await self._each(engines, "pause")
                state = S_PAUSED

            def upd(r):
                r.iro_state, r.engines, r.removed_endpoints = state, names, removed
                r.conditions["EngineReadyForRecovery"] = "True"
                r.message = "; ".join(errs)
            self.store.update(rr.name, upd)
            log.info("RecoveryRequest %s (%s, track %s): engines %s -> %s", rr.name, rr.requested_action,
                     rr.track, names, state)
            return
        if rr.phase == "Completed" and rr.iro_state in (S_PAUSED, S_SCALED_DOWN, S_NEW):
            errs = await self._each(engines, "scale_up" if rr.iro_state == S_SCALED_DOWN else "resume")
            ok = not errs and await self._wait_healthy(engines)
            if not ok and not errs:  # still faulted after the recovery: one retry, then give up
                errs += await self._each(engines, "retry")
                ok = not errs and await self._wait_healthy(engines)
            if ok:
                self.restore_routing(rr.removed_endpoints)
            else:
                self.remove_from_routing(engines)

            def upd(r):
                r.iro_state = S_RECOVERED if ok else S_DEGRADED
                r.message = "; ".join(errs) or ("" if ok else "engine not healthy after recovery")
                if ok:
                    r.removed_endpoints = []
            self.store.update(rr.name, upd)
            log.info("RecoveryRequest %s: %s", rr.name, "recovered" if ok else "degraded")
            return
        if rr.phase == "Failed":
            removed = rr.removed_endpoints + self.remove_from_routing(engines)

            def upd(r):
                r.iro_state, r.removed_endpoints = S_DEGRADED, removed
                r.message = "infrastructure recovery failed; engines kept out of routing"
            self.store.update(rr.name, upd)
            log.warning("RecoveryRequest %s failed: %s out of routing", rr.name, names)

    def _covered(self, a: EngineAdapter) -> bool:
        return any(rr.active and (a.name in rr.engines or a in self.affected(rr)) for rr in self.store.list())

    async def on_engine_fault(self, a: EngineAdapter, ev: dict):
        """Engine-initiated channel: transient unless a RecoveryRequest covers it."""
        if ev.get("action") not in (None, "detected") or not ev.get("faults", True):
            return
        async with self._lock:
            if self._covered(a) or a.name in self.degraded:
                return
            now = time.monotonic()
            q = self.transient[a.name]
            q.append(now)
            while q and now - q[0] > self.retry_window:
                q.popleft()
            if len(q) > self.max_retries:
                log.warning("engine %s: %d faults in %.0fs, taking it out of routing", a.name, len(q),
                            self.retry_window)
                self.degraded.add(a.name)
                self.degraded_eps[a.name] = self.remove_from_routing([a])
                return
            try:
                await self._do(a, "retry")
            except Exception as e:  # noqa: BLE001
                log.warning("engine %s: retry failed: %s", a.name, e)

    def readmit(self, name: str):
        """Operator action: put an engine IRO gave up on back into routing."""
        self.degraded.discard(name)
        self.transient.pop(name, None)
        self.restore_routing(self.degraded_eps.pop(name, []))

    async def reconcile(self):
        async with self._lock:
            for rr in self.store.list():
                try:
                    await self.reconcile_one(rr)
                except Exception:  # noqa: BLE001
                    log.exception("reconcile %s", rr.name)
        if self.poll_status:  # fallback for engines without an event channel
            for a in self.adapters:
                st = await a.status()
                faulted = st.get("status") in ("faulted", "unreachable")
                if faulted and a.name not in self._faulted:
                    await self.on_engine_fault(a, {"action": "detected", "faults": st.get("faults")})
                (self._faulted.add if faulted else self._faulted.discard)(a.name)

    async def _loop(self):
        while True:
            await self.reconcile()
            await asyncio.sleep(self.interval)

    def start(self):
        loop = asyncio.get_running_loop()
        for a in self.adapters:
            s = a.fault_events(lambda ad, ev: loop.create_task(self.on_engine_fault(ad, ev)))
            if s is not None:
                self._subs.append(s)
        self._task = loop.create_task(self._loop())
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
        for s in self._subs:
            await s.stop()

    # ---------------------------------------------------------- HTTP
    def render_metrics(self) -> str:
        lines = ["# HELP iro_recovery_requests RecoveryRequest objects by phase and IRO state",
                 "# TYPE iro_recovery_requests gauge"]
        cnt = defaultdict(int)
        for rr in self.store.list():
            cnt[(rr.phase, rr.iro_state or "New", rr.requested_action)] += 1
        for (ph, st, act), n in sorted(cnt.items()):
            lines.append(f'iro_recovery_requests{{phase="{ph}",iro_state="{st}",requested_action="{act}"}} {n}')
        lines += ["# HELP iro_engine_actions_total Engine adapter operations issued",
                  "# TYPE iro_engine_actions_total counter"]
        for (eng, act), n in sorted(self.actions.items()):
            lines.append(f'iro_engine_actions_total{{engine="{eng}",action="{act}"}} {n}')
        lines += ["# HELP iro_engine_degraded Engines taken out of routing after repeated transient faults",
                  "# TYPE iro_engine_degraded gauge"]
        for a in self.adapters:
            lines.append(f'iro_engine_degraded{{engine="{a.name}"}} {int(a.name in self.degraded)}')
        return "\n".join(lines) + "\n"

    def app(self) -> web.Application:
        app = web.Application()

        async def healthz(_):
            return web.Response(text="ok")

        async def metrics(_):
            return web.Response(text=self.render_metrics(), content_type="text/plain")

        async def list_rr(_):
            return web.json_response({"items": [rr.to_obj() for rr in self.store.list()]})

        async def create_rr(req):
            try:
                rr = self.store.create(await req.json())
            except FileExistsError as e:
                return web.json_response({"error": f"{e} exists"}, status=409)
            except (ValueError, KeyError, TypeError) as e:
                return web.json_response({"error": str(e)}, status=400)
            return web.json_response(rr.to_obj(), status=201)

        async def get_rr(req):
            rr = self.store.get(req.match_info["name"])
            return web.json_response(rr.to_obj()) if rr else web.json_response({"error": "not found"}, status=404)

        async def patch_status(req):
            body = await req.json()
            try:
                rr = self.store.set_phase(req.match_info["name"], (body.get("status") or body).get("phase"))
            except ValueError as e:
                return web.json_response({"error": str(e)}, status=400)
            if rr is None:
                return web.json_response({"error": "not found"}, status=404)
            return web.json_response(rr.to_obj())

        async def readmit(req):
            self.readmit(req.match_info["engine"])
            return web.json_response({"readmitted": req.match_info["engine"]})

        r = app.router
        r.add_get("/healthz", healthz)
        r.add_get("/metrics", metrics)
        r.add_get("/apis/recoveryrequests", list_rr)
        r.add_post("/apis/recoveryrequests", create_rr)
        r.add_get("/apis/recoveryrequests/{name}", get_rr)
        r.add_patch("/apis/recoveryrequests/{name}/status", patch_status)
        r.add_post("/engines/{engine}/readmit", readmit)
        return app


# ------------------------------------------------------------------ CLI
def main(argv=None):
    p = argparse.ArgumentParser("llmd-amd resilience operator")
    sub = p.add_subparsers(dest="cmd")
    run = sub.add_parser("run", help="run the operator (default)")
    for q in (p, run):
        q.add_argument("--config")
        q.add_argument("--port", type=int, default=8480)
        q.add_argument("--log-level", default="info")
    rq = sub.add_parser("request", help="create a RecoveryRequest (infrastructure side)")
    rq.add_argument("--store", required=True)
    rq.add_argument("--node", required=True)
    rq.add_argument("--device", type=int)
    rq.add_argument("--action", required=True, choices=sorted(TRACKS))
    rq.add_argument("--error-code")
    rq.add_argument("--name")
    cp = sub.add_parser("complete", help="mark a RecoveryRequest Completed (or Failed)")
    cp.add_argument("--store", required=True)
    cp.add_argument("name")
    cp.add_argument("--failed", action="store_true")
    a = p.parse_args(argv)
    if a.cmd == "request":
        spec = {"nodeName": a.node, "requestedAction": a.action}
        if a.device is not None:
            spec["deviceID"] = a.device
        if a.error_code:
            spec["errorCode"] = a.error_code
        rr = RecoveryStore(a.store).create({"metadata": {"name": a.name} if a.name else {}, "spec": spec})
        print(rr.name)
        return
    if a.cmd == "complete":
        if RecoveryStore(a.store).set_phase(a.name, "Failed" if a.failed else "Completed") is None:
            raise SystemExit(f"no RecoveryRequest {a.name}")
        return
    if not a.config:
        p.error("--config is required")
    logging.basicConfig(level=a.log_level.upper(), format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    with open(a.config) as f:
        cfg = yaml.safe_load(f) or {}

    async def _run():
        op = ResilienceOperator(cfg).start()
        runner = web.AppRunner(op.app())
        await runner.setup()
        await web.TCPSite(runner, "0.0.0.0", a.port).start()
        log.info("IRO: %d engines, store %s, API on :%d", len(op.adapters), op.store.root, a.port)
        try:
            await asyncio.Event().wait()
        finally:
            await op.stop()
            await runner.cleanup()

    asyncio.run(_run())


if __name__ == "__main__":
    main()
