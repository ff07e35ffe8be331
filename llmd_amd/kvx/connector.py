"""Scheduler-facing KV connector (``--kv-transfer-config``).

Config (vLLM-compatible keys): ``{"kv_connector": "KvxConnector" |
"NixlConnector", "kv_role": "kv_producer" | "kv_consumer" | "kv_both",
"kv_load_failure_policy": "recompute" | "fail", "kv_connector_extra_config":
{"transport": "auto" | "ipc" | "dma" | "tcp", "side_channel_port": 5557,
"abort_timeout": 480, "require_ipc": false}}``. ``require_ipc``: a GPU pull
that cannot use the xGMI IPC/VMM path fails (counted in
vllm:nixl_num_failed_transfers) instead of degrading to TCP; bench.py sets it.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

from .agent import KvxAgent

log = logging.getLogger("llmd.kvx.connector")


class KvxMetrics:
    """NIXL-compatible metric names so the P/D dashboards work unchanged."""

    def __init__(self, model: str):
        r = self.reg = CollectorRegistry()
        L = ["model_name"]
        self.model = model
        self.xfer = Histogram("vllm:nixl_xfer_time_seconds", "KV transfer time", L,
                              buckets=(.001, .002, .005, .01, .02, .05, .1, .2, .5, 1, 2, 5), registry=r)
        self.bytes = Histogram("vllm:nixl_bytes_transferred", "Bytes per transfer", L,
                               buckets=tuple(2 ** i for i in range(16, 36, 2)), registry=r)
        self.post = Histogram("vllm:nixl_post_time_seconds", "Transfer post time", L,
                              buckets=(.0001, .0005, .001, .005, .01, .05), registry=r)
        self.desc = Histogram("vllm:nixl_num_descriptors", "Descriptors (blocks) per transfer", L,
                              buckets=(1, 4, 16, 64, 256, 1024, 4096), registry=r)
        self.failed = Counter("vllm:nixl_num_failed_transfers", "Failed transfers", L, registry=r)
        # pulls that left the xGMI IPC path for the TCP fallback (0 on a healthy node)
        self.ipc_fallback = Counter("llmd:kvx_ipc_fallback", "Pulls degraded from IPC to TCP", L, registry=r)
        self.striped = Counter("llmd:kvx_striped_pulls", "Pulls striped over the direct link + relays", L,
                               registry=r)
        self.n_striped = 0
        self.n_failed = 0
        self.n_ipc_fallback = 0

    def observe(self, ok: bool, dt: float, nbytes: int, nblocks: int):
        m = self.model
        if not ok:
            self.failed.labels(m).inc()
            self.n_failed += 1
            return
        self.xfer.labels(m).observe(dt)
        self.bytes.labels(m).observe(nbytes)
        self.desc.labels(m).observe(nblocks)

    def on_striped(self, paths: int):
        self.striped.labels(self.model).inc()
        self.n_striped += 1

    def on_ipc_fallback(self):
        self.ipc_fallback.labels(self.model).inc()
        self.n_ipc_fallback += 1

    def render(self) -> bytes:
        return generate_latest(self.reg)


class KvxConnector:
    def __init__(self, cfg, engine):
        kt = cfg.kv_transfer_config or {}
        extra = kt.get("kv_connector_extra_config") or {}
        self.engine = engine
        self.role = kt.get("kv_role", "kv_both")
        self.failure_policy = kt.get("kv_load_failure_policy", "recompute")
        self.metrics = KvxMetrics(cfg.served_name)
        from llmd_amd.parallel.state import get_state

        st = get_state()
        self.agent = KvxAgent(engine.runner.kv, vmm=getattr(engine.runner, "vmm", None),
                              kv_swa=getattr(engine.runner, "kv_swa", None),
                              host=extra.get("side_channel_host"),
                              port=int(extra.get("side_channel_port", 0) or 0),
                              tp_rank=st.tp_rank, tp_size=st.tp_size,
                              abort_timeout=float(extra.get("abort_timeout",
                                                            os.environ.get("VLLM_NIXL_ABORT_REQUEST_TIMEOUT", 480))),
                              transport=extra.get("transport", "auto"), metrics=self.metrics,
                              exports=self.role != "kv_consumer",
                              require_ipc=bool(extra.get("require_ipc", False)),
                              relays=extra.get("relays"), stripe_min_bytes=extra.get("stripe_min_bytes"))
        self._results: dict[str, bool] = {}
        self._finished: list[str] = []
        self._outputs = []
        self.tp_size = st.tp_size
        self._tp_cmds: list = []  # loads / cancels for the TP followers (flush_tp)

    # ---------------- decode side (scheduler hooks)
    def start_load(self, req, local_blocks: list):
        prm = req.kv_transfer_params or {}
        swa = getattr(local_blocks, "swa", None)
        self.agent.start_load(req.request_id, prm, local_blocks, local_swa=swa)
        if self.tp_size > 1:
            self._tp_cmds.append(("load", req.request_id, dict(prm), list(local_blocks), swa))

    def cancel_load(self, request_id: str):
        """The request was aborted while its pull is queued or running. A queued
        pull is skipped (the prefiller is still told to free its blocks); a
        running one completes. Either way the id is reported through
        ``poll_finished_recv`` so the scheduler can release the local blocks
        only once nothing writes into them any more."""
        self.agent.cancel(request_id)
        if self.tp_size > 1:
            self._tp_cmds.append(("cancel", request_id))

    def flush_tp(self):
        """TP driver, once per engine step after scheduling: forward this step's
        loads and cancels to the followers over the step-plan channel (every
        TP rank pulls its own KV-head slice; see kvx/agent.py)."""
        if not self._tp_cmds:
            return
        from llmd_amd.parallel.comm import tp_broadcast_plan

        cmds, self._tp_cmds = self._tp_cmds, []
        tp_broadcast_plan({"kvx_cmd": cmds, "driver": (self.agent.host, self.agent.port)})

    def poll_finished_recv(self) -> list[str]:
        for rid, ok in self.agent.poll_done():
            self._results[rid] = ok
            self._finished.append(rid)
        out, self._finished = self._finished, []
        return out

    def recv_ok(self, rid: str) -> bool:
        return self._results.pop(rid, False)

    # ---------------- prefill side
    def hold_for_remote(self, req, blocks: list):
        if not blocks:
            self.engine.bm.free(req.seq_id)
            return
        req.extra["kv_transfer_params_out"] = self.agent.hold(req.request_id, req.seq_id, blocks,
                                                              req.num_prompt_tokens,
                                                              swa_blocks=getattr(blocks, "swa", None))

    def tick(self):
        for h in self.agent.expired_or_freed():
            self.engine.bm.free(h.seq_id)

    def take_outputs(self):
        out, self._outputs = self._outputs, []
        return out

    def render_metrics(self) -> bytes:
        return self.metrics.render()

    def close(self):
        self.agent.close()


class KvxFollower:
    """A decode TP follower's half of the connector: pulls its KV-head slice
    for the loads its driver forwards and reports back (engine/tp_worker.py)."""

    def __init__(self, cfg, runner):
        kt = cfg.kv_transfer_config or {}
        extra = kt.get("kv_connector_extra_config") or {}
        from llmd_amd.parallel.state import get_state

        st = get_state()
        if kt.get("kv_role", "kv_both") != "kv_consumer":
            raise NotImplementedError("kvx with TP > 1 is supported on the decode (kv_consumer) side")
        self.agent = KvxAgent(runner.kv, vmm=getattr(runner, "vmm", None), host=extra.get("side_channel_host"),
                              kv_swa=getattr(runner, "kv_swa", None),
                              tp_rank=st.tp_rank, tp_size=st.tp_size,
                              abort_timeout=float(extra.get("abort_timeout", 480)),
                              transport=extra.get("transport", "auto"), exports=False)

    def apply(self, pl: dict):
        drv = tuple(pl["driver"])
        for c in pl["kvx_cmd"]:
            if c[0] == "load":
                self.agent.start_load(c[1], c[2], c[3], report=drv, local_swa=c[4] if len(c) > 4 else None)
            elif c[0] == "cancel":
                self.agent.cancel(c[1])

    def close(self):
        self.agent.close()


def make_connector(cfg, engine) -> Optional[KvxConnector]:
    kt = cfg.kv_transfer_config or {}
    name = kt.get("kv_connector", "KvxConnector")
    if name in ("KvxConnector", "NixlConnector", "kvx"):
        return KvxConnector(cfg, engine)
    raise ValueError(f"unsupported kv_connector {name!r}")
